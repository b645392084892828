# H2D staging buckets (staged vs serial), smj_app buckets on the bundled CSVs, PMC traffic passes, SQ counters
set -o pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 600 python tools/h2d_overlap.py > gpurun_out/r02m/h2d_overlap.json 2> gpurun_out/r02m/h2d_overlap.err && \
python - <<'PY' > gpurun_out/r02m/smj_app_buckets.txt 2>&1
import gzip, os, shutil, subprocess, tempfile
d = tempfile.mkdtemp()
for n in ("data1.csv", "data2.csv"):
    with gzip.open(f"tests/golden/{n}.gz") as g, open(os.path.join(d, n), "wb") as f:
        shutil.copyfileobj(g, f)
for mode in ("1", "0"):
    for rep in range(3):
        r = subprocess.run(["pim-sort-merge-join_amd/bin/smj_app", os.path.join(d, "data1.csv"), os.path.join(d, "data2.csv"),
                            "-o", os.path.join(d, "result.csv")], env=dict(os.environ, SMJ_STAGED=mode),
                           capture_output=True, text=True, check=True, timeout=120)
        print(f"SMJ_STAGED={mode} run {rep}:", " | ".join(l.strip() for l in r.stdout.splitlines() if l.strip()))
PY
bash tools/gpu_run.sh r02m pmcf pmcw pmcsq
echo rc=$? >> gpurun_out/r02m/h2d_overlap.err
