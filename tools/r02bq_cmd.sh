# nontemporal loads: part_a's input rows / the pipelined part_b's gathers, same-box A/B against the base build
set -o pipefail
bash tools/ab.sh r02bq base pant pbnt
