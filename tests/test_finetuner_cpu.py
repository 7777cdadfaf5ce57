"""BASELINE config 1 plumbing: the causal-LM finetuner CLI end to end on CPU
(dataset -> train -> checkpoint-N -> resume -> final/ + .ready.txt), plus the
flag machinery and the tokenized-dataset format."""
import argparse
import os
from decimal import Decimal

import pytest
import torch

from kubernetes_cloud_amd.config.flags import DashParser, FuzzyBoolAction, validation as val
from kubernetes_cloud_amd.data.tokenized import TokenizedDataset, collate, dataset_filename, write_tokens
from kubernetes_cloud_amd.io.checkpoint import find_last_checkpoint

from .helpers import make_model_dir, make_tokens, read_jsonl


def test_dash_parser_aliases_and_help():
    p = DashParser()
    p.add_argument("--run-name")
    p.add_argument("--context_size", type=int, default=3)
    a = p.parse_args(["--run_name", "x", "--context-size", "7"])
    assert a.run_name == "x" and a.context_size == 7
    a = p.parse_args(["--run-name=y", "--context_size=9"])
    assert a.run_name == "y" and a.context_size == 9
    h = p.format_help()
    assert "--run-name" in h and "--run_name" not in h and "--context-size" in h
    # prefix abbreviation is not ambiguous between the two spellings of one flag
    a = p.parse_args(["--run", "z"])
    assert a.run_name == "z"


@pytest.mark.parametrize("argv,expected", [([], True), (["--no-resume"], False),
                                            (["--no-resume=false"], True), (["--no-resume", "0"], True),
                                            (["--no-resume=YES"], False), (["--no_resume=f"], True)])
def test_fuzzy_bool_inverted(argv, expected):
    p = DashParser()
    p.add_argument("--no-resume", action=FuzzyBoolAction, dest="resume", default=True)
    assert p.parse_args(argv).resume is expected


def test_validators(tmp_path):
    pos = val.positive(int, special_val=-1)
    assert pos("3") == 3 and pos("-1") == -1
    with pytest.raises(argparse.ArgumentTypeError):
        pos("0")
    r = val.at_most_1(val.non_negative(Decimal))
    assert r("0.9") == Decimal("0.9")
    with pytest.raises(argparse.ArgumentTypeError):
        r("1.5")
    with pytest.raises(argparse.ArgumentTypeError):
        val.at_most_32_bit(int)(str(1 << 32))
    f = tmp_path / "f"
    f.write_text("x")
    assert val.extant_file(str(f)) == str(f)
    assert val.optional_extant_file("") == ""
    with pytest.raises(argparse.ArgumentTypeError):
        val.extant_file(str(tmp_path))


def test_tokenized_dataset_padding(tmp_path):
    p = str(tmp_path / "d.tokens")
    write_tokens(p, list(range(1, 20)), 8, pad_id=0)   # 3 contexts, last padded
    ds = TokenizedDataset(p, 8, pad_token_id=0, eos_token_id=0)
    assert len(ds) == 3
    ids, m = ds[0]
    assert ids.dtype == torch.int64 and m.all()
    ids, m = ds[2]
    assert (~m).sum() == 5 and ids[-1] == 0
    b = collate([ds[1], ds[2]])
    assert (b["labels"][1][~b["attention_mask"][1]] == -100).all()
    # unambiguous pad id: every pad masked
    ds2 = TokenizedDataset(p, 8, pad_token_id=0, eos_token_id=5)
    assert (~ds2[2][1]).sum() == 5
    assert dataset_filename("novels", "EleutherAI/gpt-j-6B", 2048, 0, "gpt2") == \
        "novels-EleutherAI_gpt_j_6B-2048-b0-gpt2.tokens"


def test_checkpoint_discovery_skips_non_numeric(tmp_path):
    for n in ("checkpoint-5", "checkpoint-20", "final", "runs", "checkpoint-x"):
        os.makedirs(tmp_path / n)
    assert find_last_checkpoint(str(tmp_path)).endswith("checkpoint-20")


def _run(argv):
    from kubernetes_cloud_amd.train.finetuner import main
    return main(argv)


def test_finetuner_end_to_end_with_resume(tmp_path):
    model = make_model_dir(str(tmp_path / "model"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=24, ctx=32)
    prompts = tmp_path / "prompts.txt"
    prompts.write_text("the quick\nkubernetes cloud\n")
    out = tmp_path / "out"
    base = ["--run-name", "t1", "--model", model, "--dataset", data, "--context-size", "32",
            "--bs", "2", "--gradients", "2", "--output-path", str(out), "--logs", str(tmp_path / "logs"),
            "--save-steps", "2", "--zero-stage", "0", "--lr", "1e-3", "--prompt-file", str(prompts),
            "--prompt-every", "3", "--prompt-tokens", "4", "--prompt-samples", "2"]
    st = _run(base + ["--max-steps", "4"])
    rd = out / "results-t1"
    assert st["global_step"] == 4
    assert (rd / "checkpoint-2" / "model.safetensors").exists()
    assert (rd / "checkpoint-4" / "trainer_state.json").exists()
    assert (rd / "checkpoint-4" / "optimizer" / "rank-00000.safetensors").exists()
    assert (rd / "final" / ".ready.txt").exists()
    assert (rd / "final" / "tokenizer.json").exists() or (rd / "final" / "tokenizer_config.json").exists()
    recs = read_jsonl(tmp_path / "logs" / "t1.metrics.jsonl")
    assert len(recs) == 4 and "perf/world_samples_per_second" in recs[0]
    losses = [r["loss"] for r in recs]
    assert losses[-1] < losses[0]
    # resume continues from checkpoint-4
    st2 = _run(base + ["--max-steps", "6"])
    assert st2["global_step"] == 6
    assert (rd / "checkpoint-6").exists()
    recs = read_jsonl(tmp_path / "logs" / "t1.metrics.jsonl")
    assert [r["step"] for r in recs][-2:] == [5, 6]
    # --no-resume restarts from scratch
    st3 = _run(base + ["--max-steps", "1", "--no-resume"])
    assert st3["global_step"] == 1


def test_finetuner_final_loadable_by_hf(tmp_path):
    from transformers import AutoModelForCausalLM, AutoTokenizer
    model = make_model_dir(str(tmp_path / "model"), preset="gpt-j-6b")
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=8, ctx=16)
    _run(["--run-name", "hf", "--model", model, "--dataset", data, "--context-size", "16", "--bs", "2",
          "--gradients", "1", "--output-path", str(tmp_path / "o"), "--logs", str(tmp_path / "l"),
          "--save-steps", "0", "--max-steps", "2"])
    final = tmp_path / "o" / "results-hf" / "final"
    hm = AutoModelForCausalLM.from_pretrained(str(final))
    tok = AutoTokenizer.from_pretrained(str(final))
    ids = tok("the quick", return_tensors="pt").input_ids
    assert hm(ids).logits.shape[-1] == hm.config.vocab_size


def test_gpt2_small_124m_cpu_step(tmp_path):
    """BASELINE.json config 1: GPT-2-small (124M) finetune on CPU, world_size=1."""
    from kubernetes_cloud_amd.io.hf import save_pretrained
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import preset
    cfg = preset("gpt2")
    m = build_model(cfg, dtype=torch.float32, seed=0)
    assert 123e6 < m.num_parameters() < 126e6
    save_pretrained(m, str(tmp_path / "gpt2"))
    from .helpers import make_tokenizer
    make_tokenizer(str(tmp_path / "gpt2"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=4, ctx=64, vocab=300)
    st = _run(["--run-name", "g", "--model", str(tmp_path / "gpt2"), "--dataset", data, "--context-size", "64",
               "--bs", "1", "--gradients", "2", "--output-path", str(tmp_path / "o"), "--logs",
               str(tmp_path / "l"), "--save-steps", "2", "--max-steps", "2", "--zero-stage", "3"])
    assert st["global_step"] == 2
    assert (tmp_path / "o" / "results-g" / "final" / ".ready.txt").exists()


def test_fault_injection_and_deterministic_resume(tmp_path):
    """kill the trainer at step 3 (KCA_FAULT_STEP), restart, and the
    resumed run from checkpoint-2 must end bit-identical to an uninterrupted run."""
    import subprocess
    import sys
    from safetensors.torch import load_file
    model = make_model_dir(str(tmp_path / "model"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=24, ctx=32)

    def args(out):
        return ["--run-name", "f", "--model", model, "--dataset", data, "--context-size", "32", "--bs", "2",
                "--gradients", "2", "--output-path", str(out), "--logs", str(out / "logs"), "--save-steps", "2",
                "--zero-stage", "0", "--lr", "1e-3", "--max-steps", "5"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "kubernetes_cloud_amd.train.finetuner"]
    env = dict(os.environ, KCA_FAULT_STEP="3", KCA_FAULT_AFTER_CKPT="1", PYTHONPATH=root)
    r = subprocess.run(cmd + args(tmp_path / "a"), env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 17, r.stderr[-2000:]
    rd = tmp_path / "a" / "results-f"
    assert (rd / "checkpoint-2").exists() and not (rd / "final").exists()
    env.pop("KCA_FAULT_STEP")
    r = subprocess.run(cmd + args(tmp_path / "a"), env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run(cmd + args(tmp_path / "b"), env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    a = load_file(str(rd / "final" / "model.safetensors"))
    b = load_file(str(tmp_path / "b" / "results-f" / "final" / "model.safetensors"))
    assert max(float((a[k].float() - b[k].float()).abs().max()) for k in a) == 0.0


def test_watchdog_catches_hung_rank_and_resume_completes(tmp_path):
    """SURVEY §5.3 failure detection: a rank that stops making progress at step 3
    (KCA_FAULT_HANG_STEP) is caught by the step watchdog (KCA_WATCHDOG_TIMEOUT),
    which writes a stack report and exits 124 so the pod restarts; the restart
    resumes from checkpoint-2 and finishes."""
    import json
    import subprocess
    import sys
    model = make_model_dir(str(tmp_path / "model"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=24, ctx=32)
    out = tmp_path / "a"
    argv = ["--run-name", "h", "--model", model, "--dataset", data, "--context-size", "32", "--bs", "2",
            "--gradients", "1", "--output-path", str(out), "--logs", str(out / "logs"), "--save-steps", "2",
            "--zero-stage", "0", "--max-steps", "4"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "kubernetes_cloud_amd.train.finetuner"]
    # adaptive deadline (load-tolerant): 2 s floor, 8x the slowest step seen, 120 s before the
    # first beat -- a slow shared CI box stretches the deadline instead of tripping it early
    env = dict(os.environ, KCA_FAULT_HANG_STEP="3", KCA_WATCHDOG_TIMEOUT="2", KCA_WATCHDOG_FACTOR="8",
               KCA_WATCHDOG_STARTUP="120", PYTHONPATH=root)
    r = subprocess.run(cmd + argv, env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 124, r.stderr[-2000:]
    rd = out / "results-h"
    rep = json.loads((rd / "watchdog-rank0.json").read_text())
    # the report is written once the beat is older than the deadline in force (rounded to ms)
    assert rep["last_step"] == 3 and rep["deadline_s"] >= 2
    assert rep["seconds_since_beat"] >= rep["deadline_s"] - 1e-3
    assert "Thread" in rep["stacks"]
    env.pop("KCA_FAULT_HANG_STEP")
    r = subprocess.run(cmd + argv, env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (rd / "final" / ".ready.txt").exists()


def test_finetuner_optimizer_offload_matches_hbm(tmp_path, monkeypatch):
    """ds_config offload_optimizer=cpu (forced with KCA_OFFLOAD_OPTIMIZER=1) runs the
    host AdamW path and lands on the same weights as the in-HBM optimizer."""
    import json
    from safetensors.torch import load_file
    model = make_model_dir(str(tmp_path / "model"))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=16, ctx=32)
    ds = tmp_path / "ds.json"
    ds.write_text(json.dumps({"zero_optimization": {"stage": 2, "offload_optimizer": {"device": "cpu"}}}))
    finals = []
    for name, force in (("a", "1"), ("b", "0")):
        monkeypatch.setenv("KCA_OFFLOAD_OPTIMIZER", force)
        out = tmp_path / name
        _run(["--run-name", "o", "--model", model, "--dataset", data, "--context-size", "32", "--bs", "2",
              "--gradients", "1", "--output-path", str(out), "--logs", str(out / "l"), "--save-steps", "0",
              "--zero-stage", "2", "--lr", "1e-3", "--max-steps", "3", "--ds-config", str(ds)])
        finals.append(load_file(str(out / "results-o" / "final" / "model.safetensors")))
    a, b = finals
    assert max(float((a[k].float() - b[k].float()).abs().max()) for k in a) < 1e-5


def test_checkpoint_complete_markers(tmp_path):
    """A process that dies right after an async save (before the next save's
    barrier removes `.incomplete`) still leaves a resumable checkpoint once every
    rank's writer wrote its done marker; a missing rank marker keeps it skipped."""
    from kubernetes_cloud_amd.io.checkpoint import checkpoint_complete, find_last_checkpoint
    for step, done in ((2, (0, 1)), (4, (0,))):
        d = tmp_path / f"checkpoint-{step}"
        d.mkdir()
        (d / ".incomplete").write_text("2")
        for r in done:
            (d / f".done-rank{r}").write_text("ok")
    assert checkpoint_complete(str(tmp_path / "checkpoint-2"))
    assert not checkpoint_complete(str(tmp_path / "checkpoint-4"))
    assert find_last_checkpoint(str(tmp_path)).endswith("checkpoint-2")


def test_finetuner_xglm_from_hf_cache_id(tmp_path):
    """a Fairseq-dense / XGLM model (finetune-workflow.yaml:22-27) given as an HF id,
    resolved in the --cache hub cache (models--org--name/snapshots/<rev>), finetuned with
    --fp16-full-eval sampling and --trust-remote-code accepted; the final dir loads in transformers."""
    from transformers import AutoModelForCausalLM
    snap = tmp_path / "cache" / "models--KoboldAI--fairseq-dense-tiny" / "snapshots" / "abc123"
    (tmp_path / "cache" / "models--KoboldAI--fairseq-dense-tiny" / "refs").mkdir(parents=True)
    (tmp_path / "cache" / "models--KoboldAI--fairseq-dense-tiny" / "refs" / "main").write_text("abc123")
    make_model_dir(str(snap), preset="xglm-564m", d_model=64, num_layers=2, attention_heads=4, ffn_dim=128,
                   max_position_embeddings=64)
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=8, ctx=16)
    prompts = tmp_path / "p.txt"
    prompts.write_text("the quick\n")
    st = _run(["--run-name", "xg", "--model", "KoboldAI/fairseq-dense-tiny", "--cache", str(tmp_path / "cache"),
               "--dataset", data, "--context-size", "16", "--bs", "2", "--gradients", "1",
               "--output-path", str(tmp_path / "o"), "--logs", str(tmp_path / "l"), "--save-steps", "0",
               "--max-steps", "2", "--trust-remote-code", "--fp16-full-eval", "--prompt-file", str(prompts),
               "--prompt-every", "1", "--prompt-tokens", "3", "--prompt-samples", "1"])
    assert st["global_step"] == 2
    final = tmp_path / "o" / "results-xg" / "final"
    hm = AutoModelForCausalLM.from_pretrained(str(final))
    assert type(hm).__name__ == "XGLMForCausalLM"


def test_finetuner_unsupported_model_type_is_explicit(tmp_path):
    import json as _json

    import pytest as _pytest

    from kubernetes_cloud_amd.models.config import UnsupportedModel
    d = tmp_path / "llama"
    d.mkdir()
    (d / "config.json").write_text(_json.dumps({"model_type": "llama", "hidden_size": 64}))
    data = make_tokens(str(tmp_path / "d.tokens"), n_ctx=4, ctx=16)
    with _pytest.raises(UnsupportedModel, match="trust-remote-code"):
        _run(["--run-name", "x", "--model", str(d), "--dataset", data, "--context-size", "16", "--bs", "2",
              "--output-path", str(tmp_path / "o"), "--logs", str(tmp_path / "l"), "--trust-remote-code"])
