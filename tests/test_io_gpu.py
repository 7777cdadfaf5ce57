"""GPU: the native weight streamer (storage -> pinned ring -> HBM) and the
driver's smoke entry point."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stream_to_device_matches(tmp_path):
    from kubernetes_cloud_amd.io.tensors import load_into_module, serialize
    from kubernetes_cloud_amd.models.causal_lm import build_model
    from kubernetes_cloud_amd.models.config import PRESETS_HF, LMConfig
    cfg = dict(PRESETS_HF["gpt-j-6b"])
    cfg.update(n_embd=512, n_layer=2, n_head=4, rotary_dim=64, vocab_size=1000)
    c = LMConfig.from_hf(cfg)
    m = build_model(c, dtype=torch.bfloat16, seed=1)
    p = str(tmp_path / "gptj.tensors")
    serialize(m, p)
    md = build_model(c, device="cuda", dtype=torch.bfloat16, seed=5)
    st = load_into_module(md, p, chunk=1 << 20, threads=4)
    assert st["bytes"] > 0 and st["gbps"] > 0
    for (k, v), (_, v2) in zip(m.state_dict().items(), md.state_dict().items()):
        assert torch.equal(v, v2.cpu()), k
    md16 = build_model(c, device="cuda", dtype=torch.float16, seed=5)
    load_into_module(md16, p, odirect=False)
    assert torch.equal(md16.wte.weight.cpu(), m.wte.weight.half())


def test_graft_smoke():
    import __graft_entry__ as ge
    ge.smoke()
