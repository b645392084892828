"""Ablation timings of the radix pass / join (SMJ_DEBUG_* bits) at C3 size."""
import os, sys, json, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))
    import torch
    from smj import ops
    n = int(os.environ.get("ROWS", "100000000"))
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    bR, bS = torch.empty_like(R), torch.empty_like(S)
    J = torch.empty((n, 3), dtype=torch.int64, device=R.device); c = torch.zeros(1, dtype=torch.int64, device=R.device)
    for it in range(4):
        if it == 1:
            ops.prof_enable(True); ops.prof_report()
        Rs = ops.select_sort(R, 0, 0, 5000, out=bR); Ss = ops.select_sort(S, 0, 0, 5000, out=bS)
        ops.join(Rs, Ss, out=J, count=c, sync=False)
    torch.cuda.synchronize()
    rep = ops.prof_report()
    k, pay = Rs[:, 0], Rs[:, 1]
    ok = bool((k[1:] >= k[:-1]).all()) and bool(((k[1:] > k[:-1]) | (pay[1:] > pay[:-1])).all())
    jn = int(c.item())
    res = {k2: round(v["ms"] / v["launches"], 4) for k2, v in rep.items()}
    res["_sorted_stable"] = ok
    res["_joined"] = jn
    res["_ms_step"] = round(sum(v["ms"] for v in rep.values()) / 3, 3)
    print(json.dumps(res))
    sys.exit(0)
CONFIGS = [{}, {"SMJ_DEBUG_PASS": "1", "SMJ_DEBUG_JOIN": "1"}, {"SMJ_DEBUG_PASS": "2"}, {"SMJ_DEBUG_PASS": "3"},
           {"SMJ_DEBUG_PASS": "4"}, {"SMJ_DEBUG_PASS": "5"}]
if len(sys.argv) > 1 and sys.argv[1] == "libs":
    CONFIGS = [{}] + [{"SMJ_LIB": os.path.join(REPO, "exp", f)} for f in sorted(os.listdir(os.path.join(REPO, "exp")))]
for env in CONFIGS:
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, __file__, "child"], env=e, capture_output=True, text=True, timeout=300)
    print(env, r.stdout.strip() or r.stderr[-2000:], flush=True)
