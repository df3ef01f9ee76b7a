import torch, sys
sys.path.insert(0, "/root/repo")
from smdistributed_modelparallel_amd.ops._ext import ext
torch.manual_seed(1)
for d in (64, 128):
    qkv = torch.randn(2, 256, 3, 4, d, device="cuda", dtype=torch.bfloat16)
    outs = [ext().attention_fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], 0.125, True, 0, None, 0.0, 0, 0)[0] for _ in range(5)]
    c = qkv.clone()
    outs += [ext().attention_fwd(c[:, :, 0], c[:, :, 1], c[:, :, 2], 0.125, True, 0, None, 0.0, 0, 0)[0] for _ in range(3)]
    print(d, [ (o.float() - outs[0].float()).abs().max().item() for o in outs])
    diff = (outs[0].float() - outs[1].float()).abs()
    if diff.max() > 0:
        idx = (diff > 0).nonzero()
        print("first diffs", idx[:10].tolist(), "count", idx.shape[0])
