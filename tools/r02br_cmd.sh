# nontemporal part_b gathers: a second same-box A/B (base vs pbnt, 2 x 2 rounds)
set -o pipefail
bash tools/ab.sh r02br base pbnt && bash tools/ab.sh r02br2 pbnt base
