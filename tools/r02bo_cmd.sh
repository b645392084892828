# the driver's launch styles on one GPU: torchrun N=1, and the RCCL loopback (a one-rank nccl group, K staged exchanges)
set -o pipefail
O=gpurun_out/r02bo; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/torchrun1.json 2> $O/torchrun1.err || { echo "torchrun rc=$?"; tail -20 $O/torchrun1.err; exit 1; }
tail -c 600 $O/torchrun1.json; echo
timeout -k 10 300 python bench.py --loopback --steps 5 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/loopback.json 2> $O/loopback.err || { echo "loopback rc=$?"; tail -20 $O/loopback.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loopback.json')); print(d['value'], d['ms_per_step'], d['config'])"
