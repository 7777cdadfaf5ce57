"""The pre-tokenized dataset format of the finetune workflow (L1 data plane).

File: flat little-endian uint16 token ids, ``len(file) / 2 / ctx`` contexts of
``ctx`` tokens (finetuner-workflow/finetuner/finetuner.py:633-695); produced by
the dataset tokenizer step (finetune-workflow.yaml:423-479) -- here by
``kubernetes_cloud_amd.data.tokenizer`` / ``csrc/tokenize``.

Padding: when pad == eos the padding is ambiguous, so only the LAST context
is masked (the packer pads only the final context); otherwise every pad id is
masked. Reads are zero-copy ``numpy.memmap`` slices.
"""
from __future__ import annotations

import os
import re

import numpy as np
import torch


class TokenizedDataset(torch.utils.data.Dataset):
    def __init__(self, path: str, context_length: int = 2048, pad_token_id: int | None = None,
                 eos_token_id: int | None = None):
        self.path = path
        self.ctx = context_length
        size = os.path.getsize(path)
        self.length = size // 2 // context_length
        self._mm = np.memmap(path, dtype="<u2", mode="r", shape=(self.length * context_length,)) \
            if self.length else None
        self.pad = pad_token_id
        self.ambiguous = pad_token_id is not None and pad_token_id == eos_token_id

    @property
    def num_tokens(self) -> int:
        return self.length * self.ctx

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int):
        if idx < 0:
            idx += self.length
        if not 0 <= idx < self.length:
            raise IndexError(idx)
        a = np.asarray(self._mm[idx * self.ctx:(idx + 1) * self.ctx], dtype=np.int64)
        ids = torch.from_numpy(a)
        if self.pad is None or (self.ambiguous and idx != self.length - 1):
            mask = torch.ones_like(ids, dtype=torch.bool)
        else:
            mask = ids != self.pad
        return ids, mask


def collate(batch):
    """(input_ids, attention_mask) pairs -> the reference collector's dict
    (finetuner.py:1030-1035); labels == input_ids, masked to -100 where the
    attention mask is False (ModifiedTrainer.compute_loss, :476-477)."""
    from ..models.causal_lm import mask_to_kv
    ids = torch.stack([b[0] for b in batch])
    mask = torch.stack([b[1] for b in batch])
    labels = ids.masked_fill(~mask, -100)
    # the attention kernels' key lengths / per-key mask, classified here on the
    # host so the model forward needs no device->host sync
    return {"input_ids": ids, "attention_mask": mask, "labels": labels, "kv_len": mask_to_kv(mask)}


def write_tokens(path: str, tokens, context_length: int | None = None, pad_id: int | None = None):
    """Write a token array as the uint16 format (padding the tail context)."""
    a = np.asarray(tokens, dtype=np.int64)
    if a.size and (a.min() < 0 or a.max() > 0xFFFF):
        raise ValueError("token ids must fit uint16")
    if context_length:
        rem = a.size % context_length
        if rem:
            if pad_id is None:
                a = a[: a.size - rem]
            else:
                a = np.concatenate([a, np.full(context_length - rem, pad_id, dtype=np.int64)])
    a.astype("<u2").tofile(path)
    return path


def dataset_filename(dataset: str, model: str, context: int, boundary_index: int, tokenizer_tag: str) -> str:
    """``{dataset}-{model with / . - -> _}-{ctx}-b{boundary}-{tag}.tokens``
    (finetune-workflow.yaml:238, the Sprig replace chain)."""
    m = re.sub(r"[/.\-]", "_", model)
    return f"{dataset}-{m}-{context}-b{boundary_index}-{tokenizer_tag}.tokens"
