"""Print the overflow flags of the tiled attention fast path for a GPT-J shape."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from kubernetes_cloud_amd.ops import _lib
from kubernetes_cloud_amd.ops.attention import _strides

B, S, H, D = 8, 2048, 16, 256
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
o = torch.empty_like(q)
lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
flags = torch.full((4 * (S // 128) * B * H,), 7, device="cuda", dtype=torch.int32)
args = [q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), *_strides(q), *_strides(k),
        *_strides(v), *_strides(o), B, S, S, H, H, D, 1, D ** -0.5]
lib = _lib.require()
fn = lib.kca_attn_fwd_tiled
fn.argtypes = [_lib.P] * 5 + [_lib.LL] * 12 + [_lib.I] * 7 + [_lib.F, _lib.P, _lib.P]
rc = fn(*args, flags.data_ptr(), _lib.stream())
torch.cuda.synchronize()
print("rc", rc, "flags sum", int(flags.sum()), "unique", flags.unique().tolist())
print("lse sample", lse[0, 0, :8].tolist(), "o finite", bool(torch.isfinite(o.float()).all()))
for _ in range(3):
    fn(*args, flags.data_ptr(), _lib.stream())
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    fn(*args, flags.data_ptr(), _lib.stream())
torch.cuda.synchronize()
print("tiled only ms", (time.perf_counter() - t) / 10 * 1e3)
