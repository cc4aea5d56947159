import torch, sys, os
sys.path.insert(0, os.getcwd())
from replicann_amd import ops
torch.manual_seed(11)
M, N, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
ta, tb = sys.argv[4][0] == 't', sys.argv[4][1] == 't'
a = (torch.randn(K, M, device='cuda') if ta else torch.randn(M, K, device='cuda')).bfloat16()
b = (torch.randn(N, K, device='cuda') if tb else torch.randn(K, N, device='cuda')).bfloat16()
bias = torch.randn(N, device='cuda').bfloat16(); res = torch.randn(M, N, device='cuda').bfloat16()
ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
def rep(name, out, r):
    d = (out.float() - r).abs() > 0.05 * (r.abs() + 1)
    nbad = int(d.sum())
    print(name, 'bad', nbad, 'of', d.numel())
    if nbad:
        rows = d.any(1).nonzero().flatten(); cols = d.any(0).nonzero().flatten()
        print('  rows', rows[:20].tolist(), '... n', len(rows), ' rows%256 set', sorted(set((rows % 256).tolist()))[:40])
        print('  cols', cols[:20].tolist(), '... n', len(cols), ' cols%256 set', sorted(set((cols % 256).tolist()))[:64])
        idx = d.nonzero()[:8].tolist()
        for i, j in idx: print('   ', i, j, float(out[i, j]), float(r[i, j]))
for it in range(2):
    rep('plain', ops.gemm(a, b, ta=ta, tb=tb, cfg=9), ref)
    rep('bias', ops.gemm(a, b, ta=ta, tb=tb, cfg=9, bias=bias), ref + bias.float())
    rep('res', ops.gemm(a, b, ta=ta, tb=tb, cfg=9, residual=res), ref + res.float())
    rep('bias+res', ops.gemm(a, b, ta=ta, tb=tb, cfg=9, bias=bias, residual=res), ref + bias.float() + res.float())
