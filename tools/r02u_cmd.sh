# SQ instruction-mix and wave-cycle passes on the current build
set -o pipefail
bash tools/pmc_sq.sh r02u
echo rc=$?
