# same-box A/B: HEAD vs both-table LSD passes (lsd2) vs + late run-length scan (late); C3 and C5
set -o pipefail
bash tools/ab2.sh r03k head lsd2 late || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03k head lsd2 late || exit 1
