"""The framework's fused HIP ops (the north star's fused softmax, bias+GeLU, LayerNorm, RoPE, plus
residual dropout and vocab cross-entropy) forward + backward at training shapes, through their
public autograd wrappers, ITERS times -- for rocprofv3 time and counter passes
(tools/gpu_r5l.sh).  Shapes: GPT-2 XL mbs 16 (T = 32768 tokens, h 1600, 4h 6400, V 50257);
the reference's fused-softmax test shape (b 4, 16 heads, s 1024, fp16) and a causal softmax at
b 8, 16 heads, s 2048; GPT-J RoPE (b 8, s 2048, 16 heads, d 256, rotary 64)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdistributed_modelparallel_amd.ops import cross_entropy as ce  # noqa: E402
from smdistributed_modelparallel_amd.ops import dropout as dr  # noqa: E402
from smdistributed_modelparallel_amd.ops import gelu  # noqa: E402
from smdistributed_modelparallel_amd.ops import layernorm as ln  # noqa: E402
from smdistributed_modelparallel_amd.ops import rope  # noqa: E402
from smdistributed_modelparallel_amd.ops import softmax as sm  # noqa: E402
from smdistributed_modelparallel_amd.ops._ext import ext  # noqa: E402

assert ext() is not None, "native extension not loaded"
T, H, I, V = 32768, 1600, 6400, 50257
bf = dict(device="cuda", dtype=torch.bfloat16)
torch.manual_seed(0)


def leaf(*shape, **kw):
    return torch.randn(*shape, **kw).requires_grad_(True)


x, res = leaf(T, H, **bf), leaf(T, H, **bf)
w, b = leaf(H, **bf), leaf(H, **bf)
z, bi = leaf(T, I, **bf), leaf(I, **bf)
s1 = leaf(4, 16, 1024, 1024, device="cuda", dtype=torch.float16)
mask = torch.rand(4, 1, 1024, 1024, device="cuda") < 0.1
s2 = leaf(8, 16, 2048, 2048, **bf)
q = leaf(8, 2048, 16, 256, **bf)
logits = leaf(T, V, **bf)
tgt = torch.randint(0, V, (T,), device="cuda")
for _ in range(int(os.environ.get("ITERS", "3"))):
    ln.layer_norm(x, w, b).float().sum().backward()
    ln.add_layer_norm(x, res, w, b, dropout_p=0.1)[0].float().sum().backward()
    gelu.bias_gelu(z, bi).float().sum().backward()
    dr.dropout_add(x, res, 0.1).float().sum().backward()
    sm.scaled_masked_softmax(s1, mask, 0.125).float().sum().backward()
    sm.scaled_causal_softmax(s2, 0.125).float().sum().backward()
    rope.apply_rotary(q, 64).float().sum().backward()
    ce.cross_entropy(logits, tgt).backward()
torch.cuda.synchronize()
print("done", flush=True)
