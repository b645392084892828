import sys, time, torch, numpy as np
sys.path.insert(0, 'pim-sort-merge-join_amd')
from smj import ops
for n in [10_000_000, 100_000_000]:
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    torch.cuda.synchronize()
    keep = R[R[:, 0] > 5000]
    print(n, 'R min', R[:,0].min().item(), 'keep min', keep[:,0].min().item(), keep.shape, flush=True)
    k = keep[:, 0].contiguous()
    s = torch.sort(k, stable=True)
    print('torch sorted?', bool((s.values[1:] >= s.values[:-1]).all()), s.values[:3].tolist(), flush=True)
    Rs = ops.select_sort(R, 0, 0, 5000)
    print('ours sorted?', bool((Rs[1:,0] >= Rs[:-1,0]).all()), Rs.shape, flush=True)
    # stability check: for equal keys, payload increasing
    eq = Rs[1:,0] == Rs[:-1,0]
    print('stable?', bool((Rs[1:,1][eq] > Rs[:-1,1][eq]).all()), flush=True)
    # numpy check on cpu
    kn = keep.cpu().numpy(); order = np.argsort(kn[:,0], kind='stable')
    print('numpy equal ours', np.array_equal(kn[order], Rs.cpu().numpy()), flush=True)
    print('torch order equal numpy', np.array_equal(s.indices.cpu().numpy(), order), flush=True)
    del R, keep, k, s, Rs
    torch.cuda.empty_cache()
