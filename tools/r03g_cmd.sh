# virtual part_a probe (parts 0..16 at C3 size); staged host path timings on HEAD (threaded D2H); loopback with the new sampler
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 300 python tools/virt_probe.py > $O/virt.out 2> $O/virt.err || { echo "virt rc=$?"; tail -20 $O/virt.err; exit 1; }
cat $O/virt.out | head -6
timeout -k 10 300 python tools/h2d_overlap.py > $O/h2d.json 2> $O/h2d.err || { echo "h2d rc=$?"; tail -20 $O/h2d.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/h2d.json'))
for k,v in d.items():
    for r in v: print(k, r)
"
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop.json 2> $O/loop.err || { echo "loop rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop.json')); print('loopback', d['ms_per_step'])"
