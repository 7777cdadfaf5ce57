"""Model configuration for the causal-LM family, read from HF ``config.json``.

The reference finetunes any HF causal LM (GPT-2 / GPT-Neo / GPT-J / GPT-NeoX /
Pythia; finetuner-workflow/finetuner/finetuner.py:808-822 via
AutoModelForCausalLM; the workflow also names Fairseq dense models,
finetune-workflow.yaml:22-27 -- HF ``model_type`` "xglm") and serves BLOOM-176B (online-inference/bloom-176b/model/
bloom.py:13). We read the same HF config files so an unchanged model directory
on the PVC works, and map them onto one native decoder implementation.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os


SUPPORTED_MODEL_TYPES = ("gpt2", "gpt_neo", "gptj", "gpt_neox", "bloom", "xglm")


class UnsupportedModel(ValueError):
    """A ``model_type`` outside the native families. The reference loads any
    ``AutoModelForCausalLM`` (with ``--trust-remote-code`` for Hub code,
    finetuner.py:795-822); this framework runs its own kernels, so remote model
    code is never executed -- the error names what is supported."""

    def __init__(self, model_type: str):
        super().__init__(
            f"unsupported model_type {model_type!r}: the MI355X-native model families are "
            f"{', '.join(SUPPORTED_MODEL_TYPES)} (GPT-2, GPT-Neo, GPT-J, GPT-NeoX/Pythia, BLOOM, XGLM/fairseq-dense). "
            "--trust-remote-code cannot add an architecture: remote modeling code is not executed; "
            "convert the checkpoint to one of these families")
        self.model_type = model_type


@dataclasses.dataclass
class LMConfig:
    arch: str                      # gptj | gpt2 | gpt_neox | gpt_neo | bloom | xglm
    vocab_size: int
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int | None = None
    ffn: int | None = None
    max_pos: int = 2048
    rotary_dim: int = 0            # dims rotated per head (0: none)
    rotary_interleaved: bool = True
    rotary_base: float = 10000.0
    parallel_residual: bool = False   # GPT-J / NeoX: h + attn(ln(h)) + mlp(ln'(h))
    shared_ln: bool = False           # GPT-J uses ONE LN for both branches
    learned_pos: bool = False         # GPT-2 / GPT-Neo wpe
    alibi: bool = False               # BLOOM
    embed_ln: bool = False            # BLOOM word_embeddings_layernorm
    qkv_bias: bool = False
    out_bias: bool = False
    mlp_bias: bool = True
    lm_head_bias: bool = False
    tie_embeddings: bool = False
    gelu_approx: str = "tanh"         # "tanh" | "none"
    ln_eps: float = 1e-5
    attn_scale: float | None = None   # None -> 1/sqrt(head_dim); GPT-Neo uses 1.0
    local_window: int = 0             # GPT-Neo local attention window
    embed_scale: float = 1.0          # XGLM / fairseq-dense: token embeddings x sqrt(d_model)
    sinusoidal_pos: bool = False      # XGLM / fairseq-dense: fixed sinusoidal positions
    pos_offset: int = 0               # ... at position + 2 (fairseq padding_idx convention)
    attention_layers: tuple | None = None
    bos_token_id: int = 50256
    eos_token_id: int = 50256
    pad_token_id: int | None = None
    hf: dict = dataclasses.field(default_factory=dict, repr=False)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.n_heads

    @property
    def kv_heads(self) -> int:
        return self.n_kv_heads or self.n_heads

    @property
    def ffn_dim(self) -> int:
        return self.ffn or 4 * self.hidden

    def n_params(self) -> int:
        d, L, V, f = self.hidden, self.n_layers, self.vocab_size, self.ffn_dim
        per_layer = 4 * d * d + 2 * d * f + f + d + (4 if not self.shared_ln else 2) * d
        emb = V * d + (self.max_pos * d if self.learned_pos else 0)
        head = 0 if self.tie_embeddings else V * d + (V if self.lm_head_bias else 0)
        return L * per_layer + emb + head + 2 * d

    def flops_per_token(self, seq: int) -> float:
        """Training FLOPs/token (fwd+bwd = 3x fwd): 6N + 12*L*d*S (attention)."""
        n = self.n_params() - self.vocab_size * self.hidden * (0 if self.tie_embeddings else 1)
        n += self.vocab_size * self.hidden  # LM head matmul counts once
        return 6.0 * n + 12.0 * self.n_layers * self.hidden * seq

    @classmethod
    def from_hf(cls, cfg: dict) -> "LMConfig":
        mt = cfg.get("model_type", "")
        if mt == "gptj":
            d = cfg["n_embd"]
            return cls(arch="gptj", vocab_size=cfg["vocab_size"], hidden=d, n_layers=cfg["n_layer"],
                       n_heads=cfg["n_head"], ffn=cfg.get("n_inner") or 4 * d,
                       max_pos=cfg.get("n_positions", 2048), rotary_dim=cfg.get("rotary_dim") or d // cfg["n_head"],
                       rotary_interleaved=True, parallel_residual=True, shared_ln=True,
                       mlp_bias=True, lm_head_bias=True, gelu_approx="tanh",
                       ln_eps=cfg.get("layer_norm_epsilon", 1e-5),
                       bos_token_id=cfg.get("bos_token_id", 50256), eos_token_id=cfg.get("eos_token_id", 50256),
                       tie_embeddings=cfg.get("tie_word_embeddings", False), hf=cfg)
        if mt == "gpt2":
            d = cfg["n_embd"]
            return cls(arch="gpt2", vocab_size=cfg["vocab_size"], hidden=d, n_layers=cfg["n_layer"],
                       n_heads=cfg["n_head"], ffn=cfg.get("n_inner") or 4 * d,
                       max_pos=cfg.get("n_positions", 1024), learned_pos=True, qkv_bias=True,
                       out_bias=True, tie_embeddings=True, gelu_approx="tanh",
                       ln_eps=cfg.get("layer_norm_epsilon", 1e-5),
                       bos_token_id=cfg.get("bos_token_id", 50256), eos_token_id=cfg.get("eos_token_id", 50256),
                       hf=cfg)
        if mt == "gpt_neox":
            d = cfg["hidden_size"]
            hd = d // cfg["num_attention_heads"]
            rp = cfg.get("rope_parameters") or {}
            rot_pct = cfg.get("rotary_pct", rp.get("partial_rotary_factor", 0.25))
            rot_base = cfg.get("rotary_emb_base", rp.get("rope_theta", cfg.get("rope_theta", 10000)))
            act = cfg.get("hidden_act", "gelu")
            return cls(arch="gpt_neox", vocab_size=cfg["vocab_size"], hidden=d,
                       n_layers=cfg["num_hidden_layers"], n_heads=cfg["num_attention_heads"],
                       ffn=cfg.get("intermediate_size", 4 * d),
                       max_pos=cfg.get("max_position_embeddings", 2048),
                       rotary_dim=int(hd * rot_pct), rotary_interleaved=False,
                       rotary_base=rot_base,
                       parallel_residual=cfg.get("use_parallel_residual", True), qkv_bias=True,
                       out_bias=True, mlp_bias=True,
                       gelu_approx="none" if act == "gelu" else "tanh",
                       ln_eps=cfg.get("layer_norm_eps", 1e-5),
                       tie_embeddings=cfg.get("tie_word_embeddings", False),
                       bos_token_id=cfg.get("bos_token_id", 0), eos_token_id=cfg.get("eos_token_id", 0),
                       hf=cfg)
        if mt == "gpt_neo":
            d = cfg["hidden_size"]
            layers = []
            for kinds, n in cfg.get("attention_types", [[["global", "local"], cfg["num_layers"] // 2]]):
                layers += list(kinds) * n
            return cls(arch="gpt_neo", vocab_size=cfg["vocab_size"], hidden=d, n_layers=cfg["num_layers"],
                       n_heads=cfg["num_heads"], ffn=cfg.get("intermediate_size") or 4 * d,
                       max_pos=cfg.get("max_position_embeddings", 2048), learned_pos=True,
                       out_bias=True, tie_embeddings=True, attn_scale=1.0,
                       local_window=cfg.get("window_size", 256), attention_layers=tuple(layers),
                       gelu_approx="tanh", ln_eps=cfg.get("layer_norm_epsilon", 1e-5),
                       bos_token_id=cfg.get("bos_token_id", 50256), eos_token_id=cfg.get("eos_token_id", 50256),
                       hf=cfg)
        if mt == "bloom":
            d = cfg.get("hidden_size", cfg.get("n_embed"))
            return cls(arch="bloom", vocab_size=cfg["vocab_size"], hidden=d, n_layers=cfg.get("n_layer", cfg.get("num_hidden_layers")),
                       n_heads=cfg.get("n_head", cfg.get("num_attention_heads")), ffn=4 * d, max_pos=2048,
                       alibi=True, embed_ln=True, qkv_bias=True, out_bias=True, mlp_bias=True,
                       tie_embeddings=True, gelu_approx="tanh",
                       ln_eps=cfg.get("layer_norm_epsilon", 1e-5),
                       bos_token_id=cfg.get("bos_token_id", 1), eos_token_id=cfg.get("eos_token_id", 2),
                       pad_token_id=cfg.get("pad_token_id", 3), hf=cfg)
        if mt == "xglm":  # XGLM and the KoboldAI fairseq-dense conversions
            d = cfg["d_model"]
            act = cfg.get("activation_function", "gelu")
            return cls(arch="xglm", vocab_size=cfg["vocab_size"], hidden=d, n_layers=cfg["num_layers"],
                       n_heads=cfg["attention_heads"], ffn=cfg.get("ffn_dim", 4 * d),
                       max_pos=cfg.get("max_position_embeddings", 2048), sinusoidal_pos=True, pos_offset=2,
                       embed_scale=math.sqrt(d) if cfg.get("scale_embedding", True) else 1.0,
                       qkv_bias=True, out_bias=True, mlp_bias=True,
                       tie_embeddings=cfg.get("tie_word_embeddings", True),
                       gelu_approx="none" if act == "gelu" else "tanh", ln_eps=1e-5,
                       bos_token_id=cfg.get("bos_token_id", 0), eos_token_id=cfg.get("eos_token_id", 2),
                       pad_token_id=cfg.get("pad_token_id", 1), hf=cfg)
        raise UnsupportedModel(mt)

    @classmethod
    def from_pretrained(cls, path: str) -> "LMConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_hf(json.load(f))

    def to_hf(self) -> dict:
        if self.hf:
            return dict(self.hf)
        return PRESETS_HF.get(self.arch, {})


# Public HF configs of the models the reference names -- used
# for random-init benchmarking when no model directory is on disk.
PRESETS_HF: dict = {
    "gpt2": {"model_type": "gpt2", "vocab_size": 50257, "n_embd": 768, "n_layer": 12, "n_head": 12,
             "n_positions": 1024, "layer_norm_epsilon": 1e-5, "bos_token_id": 50256, "eos_token_id": 50256,
             "architectures": ["GPT2LMHeadModel"], "activation_function": "gelu_new"},
    "gpt2-xl": {"model_type": "gpt2", "vocab_size": 50257, "n_embd": 1600, "n_layer": 48, "n_head": 25,
                "n_positions": 1024, "layer_norm_epsilon": 1e-5, "bos_token_id": 50256, "eos_token_id": 50256,
                "architectures": ["GPT2LMHeadModel"], "activation_function": "gelu_new"},
    "gpt-j-6b": {"model_type": "gptj", "vocab_size": 50400, "n_embd": 4096, "n_layer": 28, "n_head": 16,
                 "n_positions": 2048, "rotary_dim": 64, "n_inner": None, "layer_norm_epsilon": 1e-5,
                 "bos_token_id": 50256, "eos_token_id": 50256, "tie_word_embeddings": False,
                 "architectures": ["GPTJForCausalLM"], "activation_function": "gelu_new"},
    "pythia-2.8b": {"model_type": "gpt_neox", "vocab_size": 50304, "hidden_size": 2560,
                    "num_hidden_layers": 32, "num_attention_heads": 32, "intermediate_size": 10240,
                    "max_position_embeddings": 2048, "rotary_pct": 0.25, "rotary_emb_base": 10000,
                    "use_parallel_residual": True, "hidden_act": "gelu", "layer_norm_eps": 1e-5,
                    "bos_token_id": 0, "eos_token_id": 0, "tie_word_embeddings": False,
                    "architectures": ["GPTNeoXForCausalLM"]},
    "gpt-neox-20b": {"model_type": "gpt_neox", "vocab_size": 50432, "hidden_size": 6144,
                     "num_hidden_layers": 44, "num_attention_heads": 64, "intermediate_size": 24576,
                     "max_position_embeddings": 2048, "rotary_pct": 0.25, "rotary_emb_base": 10000,
                     "use_parallel_residual": True, "hidden_act": "gelu_fast", "layer_norm_eps": 1e-5,
                     "bos_token_id": 0, "eos_token_id": 0, "tie_word_embeddings": False,
                     "architectures": ["GPTNeoXForCausalLM"]},
    "bloom-176b": {"model_type": "bloom", "vocab_size": 250880, "hidden_size": 14336, "n_layer": 70,
                   "n_head": 112, "layer_norm_epsilon": 1e-5, "bos_token_id": 1, "eos_token_id": 2,
                   "pad_token_id": 3, "architectures": ["BloomForCausalLM"]},
    "xglm-564m": {"model_type": "xglm", "vocab_size": 256008, "d_model": 1024, "num_layers": 24,
                  "attention_heads": 16, "ffn_dim": 4096, "max_position_embeddings": 2048,
                  "activation_function": "gelu", "scale_embedding": True, "bos_token_id": 0, "pad_token_id": 1,
                  "eos_token_id": 2, "architectures": ["XGLMForCausalLM"]},
    "bloom-560m": {"model_type": "bloom", "vocab_size": 250880, "hidden_size": 1024, "n_layer": 24,
                   "n_head": 16, "layer_norm_epsilon": 1e-5, "bos_token_id": 1, "eos_token_id": 2,
                   "pad_token_id": 3, "architectures": ["BloomForCausalLM"]},
}


def preset(name: str, **overrides) -> LMConfig:
    cfg = dict(PRESETS_HF[name])
    cfg.update(overrides)
    return LMConfig.from_hf(cfg)
