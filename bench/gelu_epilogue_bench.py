"""GPT-J MLP GELU: the fused operand passes (ops/fused_block.py) against hipBLASLt's GELU epilogues.

GPT-J-6B training shapes (micro-batch 16 x seq 2048 = 32768 tokens, d 4096, ffn 16384, tanh GELU).
Every layout the TN weight-gradient GEMMs need is produced in both variants:

  forward   pass : u = x Wfc_in^T + b (GEMM, bias epilogue); kca_gelu_fwd_t: g and g^T
            epi  : g = gelu(x Wfc_in^T + b) with u as the epilogue's aux output (GELU_AUX_BIAS);
                   kca_transpose_bf16: g^T
  backward  pass : dg = dm Wfc_out (GEMM); kca_gelu_bwd_t: du, du^T, bias partials; column reduce
            epi  : du = (dm Wfc_out) * gelu'(u) with the bias gradient from the epilogue
                   (DGELU_BGRAD, u as aux input); kca_transpose_bf16: du^T

Both GEMM variants go through csrc/kernels/gemm_lt.hip (same candidate timing), and the torch
F.linear (TunableOp table of bench.py) time of the plain GEMM is printed beside them. Numerics:
each output against an fp32 reference of the same op. One JSON line per variant.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kubernetes_cloud_amd.ops import _lib  # noqa: E402
from kubernetes_cloud_amd.ops.linear import _WS_BYTES, _workspace  # noqa: E402


def timed(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--f", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tunableop-file", default=os.path.join(ROOT, "tuning", "tunableop_results.csv"))
    args = ap.parse_args()
    if os.path.exists(args.tunableop_file):
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.set_filename(args.tunableop_file, insert_device_ordinal=False)
        tunable.tuning_enable(False)
        tunable.read_file(args.tunableop_file)
    T, d, f = args.tokens, args.d, args.f
    assert T % 64 == 0 and d % 64 == 0 and f % 64 == 0
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bf = torch.bfloat16
    x = torch.randn(T, d, device=dev, dtype=bf)
    w_in = (torch.randn(f, d, device=dev) * d ** -0.5).to(bf)
    b_in = (torch.randn(f, device=dev) * 0.1).to(bf)
    w_out = (torch.randn(d, f, device=dev) * f ** -0.5).to(bf)
    w_out_t = w_out.t().contiguous()  # [f, d]: the fc_out TLinear's weight_t
    dm = (torch.randn(T, d, device=dev) * 0.01).to(bf)
    ws = _workspace(dev)
    st = _lib.stream()

    u = torch.empty(T, f, device=dev, dtype=bf)
    g = torch.empty_like(u)
    gt = torch.empty(f, T, device=dev, dtype=bf)
    dg = torch.empty_like(u)
    du = torch.empty_like(u)
    dut = torch.empty_like(gt)
    part = torch.empty(T // 64, f, device=dev, dtype=torch.float32)
    bgrad = torch.empty(f, device=dev, dtype=bf)
    bgrad32 = torch.empty(f, device=dev, dtype=torch.float32)

    def gemm(a, w, bias, out):
        rc = _lib.call("kca_gemm_lt", a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), _lib.ptr(bias), None, 0,
                       out.data_ptr(), out.stride(0), a.shape[0], w.shape[0], a.shape[1], 0.0, _lib.ptr(ws),
                       _WS_BYTES, st)
        assert rc == 0, rc

    def gemm_gelu(a, w, kind, bias, aux, out):
        rc = _lib.call("kca_gemm_lt_gelu", a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), kind,
                       _lib.ptr(bias), aux.data_ptr(), aux.stride(0), out.data_ptr(), out.stride(0), a.shape[0],
                       w.shape[0], a.shape[1], _lib.ptr(ws), _WS_BYTES, st)
        assert rc == 0, rc

    def fwd_pass():
        gemm(x, w_in, b_in, u)
        _lib.call("kca_gelu_fwd_t", u.data_ptr(), f, g.data_ptr(), f, gt.data_ptr(), T, T, f, 1, st)

    def fwd_epi():
        gemm_gelu(x, w_in, kf, bias_f, u, g)
        _lib.call("kca_transpose_bf16", g.data_ptr(), f, gt.data_ptr(), T, T, f, st)

    def bwd_pass():
        gemm(dm, w_out_t, None, dg)
        _lib.call("kca_gelu_bwd_t", dg.data_ptr(), f, u.data_ptr(), f, du.data_ptr(), f, dut.data_ptr(), T,
                  part.data_ptr(), T, f, 1, st)
        _lib.call("kca_col_reduce_f32", part.data_ptr(), part.shape[0], f, bgrad.data_ptr(), None, st)

    def bwd_epi():
        gemm_gelu(dm, w_out_t, kb, bgrad32, u, du)
        _lib.call("kca_transpose_bf16", du.data_ptr(), f, dut.data_ptr(), T, T, f, st)

    # ---- which epilogue configurations hipBLASLt has kernels for (kind | 4: fp32 bias, | 8: default aux type)
    b_in32 = b_in.float()
    probe = {}
    for kind, bias in ((1, b_in), (5, b_in32), (9, b_in), (13, b_in32), (1, None), (9, None), (2, bgrad32),
                       (10, bgrad32), (2, None), (10, None), (3, b_in), (3, None)):
        try:
            gemm_gelu(x, w_in, kind, bias, u, g) if kind & 3 != 2 else gemm_gelu(dm, w_out_t, kind, bias, u, du)
            probe[f"{kind}{'' if bias is not None else '_nobias'}"] = "ok"
        except (RuntimeError, AssertionError) as e:
            probe[f"{kind}{'' if bias is not None else '_nobias'}"] = str(e)[-40:]
    torch.cuda.synchronize()
    print(json.dumps(dict(variant="probe", **probe)), flush=True)
    kf = next((k for k in ("1", "5", "9", "13") if probe.get(k) == "ok"), None)
    kb = next((k for k in ("2", "10") if probe.get(k) == "ok"), None)
    if kf is None or kb is None:
        # only the aux-less GELU_BIAS epilogue exists: it cannot keep u for the backward; its cost beside
        # the bias-only GEMM is recorded for the notes
        t_b = timed(lambda: gemm(x, w_in, b_in, u), args.iters)
        t_g = timed(lambda: gemm_gelu(x, w_in, 3, b_in, u, g), args.iters)
        t_p = timed(fwd_pass, args.iters)
        print(json.dumps(dict(variant="no_aux_epilogue", T=T, d=d, f=f, lt_bias_fwd_ms=round(t_b, 4),
                              lt_gelu_bias_fwd_ms=round(t_g, 4), pass_fwd_ms=round(t_p, 4))), flush=True)
        raise SystemExit("no hipBLASLt GELU aux / DGELU epilogue kernel for these shapes (status 4: no algorithm)")
    kf, kb = int(kf), int(kb)
    bias_f = b_in32 if kf & 4 else b_in

    # ---- numerics against fp32 references (rows subsampled for the reference GEMMs)
    rows = slice(0, 2048)
    u_ref = (x[rows].float() @ w_in.float().t() + b_in.float())
    g_ref = gelu_tanh(u_ref)
    h_ref = dm.float() @ w_out_t.float().t()  # dg, all rows (the bias gradient sums over them)
    recs = []
    for name, fwd, bwd in (("pass", fwd_pass, bwd_pass), ("epi", fwd_epi, bwd_epi)):
        fwd()
        torch.cuda.synchronize()
        u_full = u.float()
        # gelu'(u) from autograd on the fp32 copy of this variant's own u
        uu = u_full.clone().requires_grad_(True)
        gelu_tanh(uu).sum().backward()
        du_ref = h_ref * uu.grad
        del uu
        num = {"g_rel": rel(g[rows], g_ref), "gt_rel": rel(gt[:, rows].t(), g_ref), "u_rel": rel(u[rows], u_ref)}
        bwd()
        torch.cuda.synchronize()
        bsum = bgrad32 if name == "epi" else bgrad.float()
        num.update(du_rel=rel(du, du_ref), dut_rel=rel(dut.t(), du_ref), bgrad_rel=rel(bsum, du_ref.sum(0)))
        del du_ref, u_full
        t_f = timed(fwd, args.iters)
        t_b = timed(bwd, args.iters)
        recs.append(dict(variant=name, fwd_ms=round(t_f, 4), bwd_ms=round(t_b, 4), **{k: round(v, 5) for k, v in num.items()}))
    t_lin_f = timed(lambda: F.linear(x, w_in, b_in), args.iters)
    t_lin_b = timed(lambda: F.linear(dm, w_out_t), args.iters)
    t_gemm_f = timed(lambda: gemm(x, w_in, b_in, u), args.iters)
    t_gemm_b = timed(lambda: gemm(dm, w_out_t, None, dg), args.iters)
    t_epi_f = timed(lambda: gemm_gelu(x, w_in, kf, bias_f, u, g), args.iters)
    t_epi_b = timed(lambda: gemm_gelu(dm, w_out_t, kb, bgrad32, u, du), args.iters)
    for r in recs:
        print(json.dumps(dict(T=T, d=d, f=f, **r)), flush=True)
    print(json.dumps(dict(T=T, d=d, f=f, variant="gemm_only", torch_linear_fwd_ms=round(t_lin_f, 4),
                          torch_linear_bwd_ms=round(t_lin_b, 4), lt_bias_fwd_ms=round(t_gemm_f, 4),
                          lt_bwd_ms=round(t_gemm_b, 4), lt_gelu_aux_fwd_ms=round(t_epi_f, 4),
                          lt_dgelu_bgrad_bwd_ms=round(t_epi_b, 4))), flush=True)


if __name__ == "__main__":
    main()
