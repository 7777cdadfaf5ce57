"""CLI flag machinery shared by every entry point.

Behavioural contract of the reference's finetuner utilities
(finetuner-workflow/finetuner/utils.py:134-356), re-implemented:

* :class:`DashParser` -- every option is reachable as ``--x-y`` *and*
  ``--x_y``; help lists only the dashed spelling; two spellings of one option
  are never reported as an ambiguous prefix.
* :class:`FuzzyBoolAction` -- ``--flag``, ``--flag=true/false/0/1/yes/no``;
  "0", "no", "f", "false" (any case) mean False (== flag absent), anything
  else True (== flag present). With ``default=True`` the meaning inverts, which
  is how ``--no-resume`` (dest=resume) and ``--no-shuffle`` work.
* :data:`validation` -- ``positive``, ``non_negative``, ``at_most_1``,
  ``at_most_32_bit`` (composable, optional ``special_val``) and
  ``extant_file`` / ``optional_extant_file``.
"""
from __future__ import annotations

import argparse
import operator
import os
import types
from functools import partial

_FALSY = {"0", "no", "f", "false"}


class _DashOnlyHelp(argparse.HelpFormatter):
    def _format_action_invocation(self, action):
        if action.option_strings:
            shown = [s for s in action.option_strings if "_" not in s.lstrip("-")] or action.option_strings[:1]
            saved = action.option_strings
            action.option_strings = shown
            try:
                return super()._format_action_invocation(action)
            finally:
                action.option_strings = saved
        return super()._format_action_invocation(action)


class DashParser(argparse.ArgumentParser):
    def __init__(self, *args, **kwargs):
        kwargs.setdefault("formatter_class", _DashOnlyHelp)
        self._canonical = {}
        super().__init__(*args, **kwargs)

    def add_argument(self, *names, **kwargs):
        if names and not names[0].startswith(tuple(self.prefix_chars)):
            # positional: argparse dests cannot contain dashes
            name = names[0].replace("-", "_")
            if "_" in name:
                kwargs.setdefault("metavar", name.replace("_", "-"))
            return super().add_argument(name, *names[1:], **kwargs)
        expanded: list[str] = []
        for n in names:
            body = n.lstrip(self.prefix_chars)
            pre = n[: len(n) - len(body)]
            dashed = pre + body.replace("_", "-")
            under = pre + body.replace("-", "_")
            for v in (dashed, n, under):
                if v not in expanded:
                    expanded.append(v)
                self._canonical[v] = dashed
        return super().add_argument(*expanded, **kwargs)

    def _get_option_tuples(self, option_string):
        tuples = super()._get_option_tuples(option_string)
        if len(tuples) <= 1:
            return tuples
        seen = {}
        for t in tuples:
            action, opt = t[0], t[1]
            key = (id(action), self._canonical.get(opt, opt))
            seen.setdefault(key, t)
        return list(seen.values())


class FuzzyBoolAction(argparse.Action):
    def __init__(self, option_strings, dest, nargs=None, default=False, type=None, choices=None,
                 required=False, help=None, metavar=None, const=None):
        if default is None:
            default = False
        if not isinstance(default, bool):
            raise ValueError("FuzzyBoolAction needs a boolean default")
        flag_value = not default

        def parse(text: str) -> bool:
            return default if text.strip().lower() in _FALSY else flag_value

        super().__init__(option_strings, dest, nargs=argparse.OPTIONAL, const=flag_value,
                         default=default, type=type or parse, choices=choices, required=required,
                         help=help, metavar=metavar or "BOOL")

    def __call__(self, parser, namespace, values, option_string=None):
        setattr(namespace, self.dest, values)


def _bounded(num_type, op, bound, what, special_val=None):
    desc = what if special_val is None else f"{what} or {special_val}"

    def check(text):
        value = num_type(text)
        if op(value, bound) or (special_val is not None and value == special_val):
            return value
        raise argparse.ArgumentTypeError(f"must be {desc}, not {value}")

    check.__name__ = f"{what.replace(' ', '_')}"
    return check


def _file(text: str, optional: bool = False) -> str:
    if not text:
        if optional:
            return ""
        raise argparse.ArgumentTypeError("must be specified")
    if os.path.isfile(text):
        return text
    if os.path.lexists(text):
        raise argparse.ArgumentTypeError(f"invalid file: {text} exists, but isn't a file")
    raise argparse.ArgumentTypeError(f"file not found: {text}")


validation = types.SimpleNamespace(
    positive=partial(lambda t, special_val=None: _bounded(t, operator.gt, 0, "positive", special_val)),
    non_negative=partial(lambda t, special_val=None: _bounded(t, operator.ge, 0, "non-negative", special_val)),
    at_most_1=partial(lambda t, special_val=None: _bounded(t, operator.le, 1, "at most 1", special_val)),
    at_most_32_bit=partial(lambda t, special_val=None: _bounded(t, operator.le, (1 << 32) - 1,
                                                               "at most 2 ** 32 - 1", special_val)),
    extant_file=_file,
    optional_extant_file=partial(_file, optional=True),
)


def bool_t(s) -> bool:
    """The SD trainer's plain ``type=bool_t`` converter (sd-finetuner/finetuner.py:48)."""
    return str(s).strip().lower() not in ("false", "0", "no", "f", "")
