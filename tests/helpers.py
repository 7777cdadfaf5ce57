"""Test fixtures: synthetic model directories, tokenizers and token files."""
from __future__ import annotations

import json
import os

import torch


def make_tokenizer(path: str, vocab_size: int = 300):
    """Train a tiny byte-level BPE (tokenizers lib) and save it HF-style."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=["<|endoftext|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = ["the quick brown fox jumps over the lazy dog",
              "kubernetes cloud on mi355x gpus with hip kernels",
              "a finetuner trains a language model on tokens"] * 20
    tok.train_from_iterator(corpus, tr)
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, eos_token="<|endoftext|>",
                                   bos_token="<|endoftext|>", unk_token="<|endoftext|>")
    fast.save_pretrained(path)
    return fast


def make_model_dir(path: str, preset: str = "gpt2", vocab_size: int = 320, tokenizer: bool = True,
                   **over):
    from kubernetes_cloud_amd.io.hf import save_pretrained
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig

    os.makedirs(path, exist_ok=True)
    cfg = dict(PRESETS_HF[preset])
    small = {"gpt2": dict(n_embd=64, n_layer=2, n_head=4, n_positions=128),
             "gpt-j-6b": dict(n_embd=64, n_layer=2, n_head=4, rotary_dim=8, n_positions=128),
             "pythia-2.8b": dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                 intermediate_size=128, max_position_embeddings=128)}.get(preset, {})
    cfg.update(small)
    cfg.update(vocab_size=vocab_size, bos_token_id=0, eos_token_id=0)
    cfg.update(over)
    m = build_model(LMConfig.from_hf(cfg), dtype=torch.float32, seed=0)
    save_pretrained(m, path)
    if tokenizer:
        make_tokenizer(path)
    return path


def make_tokens(path: str, n_ctx: int, ctx: int, vocab: int = 300, seed: int = 0, pad_id: int = 0):
    from kubernetes_cloud_amd.data.tokenized import write_tokens
    g = torch.Generator().manual_seed(seed)
    toks = torch.randint(1, vocab, (n_ctx * ctx - ctx // 2,), generator=g).tolist()
    return write_tokens(path, toks, ctx, pad_id)


def read_jsonl(path):
    with open(path) as f:
        return [json.loads(x) for x in f if x.strip()]


def make_sd_dir(path: str, res: int = 32, prediction_type: str = "epsilon"):
    """Tiny SD pipeline in the diffusers layout (random weights)."""
    import torch
    from kubernetes_cloud_amd.models.clip_text import CLIPTextConfig, build_clip_text
    from kubernetes_cloud_amd.models.schedulers import PNDMScheduler, sd_scheduler_config
    from kubernetes_cloud_amd.models.sd_pipeline import StableDiffusionPipeline
    from kubernetes_cloud_amd.models.unet import UNetConfig, build_unet
    from kubernetes_cloud_amd.models.vae import VAEConfig, build_vae
    tok = make_tokenizer(os.path.join(path, "_tok"), vocab_size=300)
    tok.pad_token = tok.eos_token
    tok.model_max_length = 16
    te = build_clip_text(CLIPTextConfig(vocab_size=len(tok), hidden_size=32, intermediate_size=64,
                                        num_hidden_layers=2, num_attention_heads=2, max_position_embeddings=16,
                                        eos_token_id=tok.eos_token_id))
    unet = build_unet(UNetConfig(block_out_channels=(32, 64, 64, 64), cross_attention_dim=32,
                                 attention_head_dim=4, norm_num_groups=8, sample_size=res // 8))
    vae = build_vae(VAEConfig(block_out_channels=(16, 32), layers_per_block=1, norm_num_groups=8,
                              sample_size=res))
    sch = PNDMScheduler.from_config(sd_scheduler_config(prediction_type))
    pipe = StableDiffusionPipeline(unet, vae, te, tok, sch)
    pipe.save_pretrained(path)
    return path


def make_images(path: str, n: int, size: int = 40, captions: bool = True):
    from PIL import Image
    import numpy as np
    os.makedirs(path, exist_ok=True)
    rng = np.random.default_rng(0)
    for i in range(n):
        a = (rng.random((size, size + 8, 3)) * 255).astype("uint8")
        Image.fromarray(a).save(os.path.join(path, f"img{i}.png"))
        if captions:
            with open(os.path.join(path, f"img{i}.txt"), "w") as f:
                f.write(f"a photo of the quick fox number {i}\n")
    return path
