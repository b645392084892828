# part_b experiment: every tile's stores retired before the next tile starts (s_waitcnt vmcnt(0)) -- what the store drain costs
set -o pipefail
bash tools/ab.sh r02ad head drain
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > gpurun_out/r02ad/loopback.json 2> gpurun_out/r02ad/loopback.err && wc -l gpurun_out/r02ad/loopback.json
