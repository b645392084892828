# re-entry baseline on HEAD: smoke, full GPU suite, C3 bench, rocprof kernel stats
set -o pipefail
bash tools/gpu_run.sh r02p smoke tests bench prof
