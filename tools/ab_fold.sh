# A/B of the folded backward tail (GPU box): bash tools/ab_fold.sh 65536 ...  (default library first, alternating)
set -e
for r in 1 2; do
  echo "== default"; timeout -k 10 120 python tools/fold_bench.py | grep fold
  for e in "$@"; do echo "== exp $e"; BCNF_AMD_LIB=build_exp/libexp$e.so timeout -k 10 120 python tools/fold_bench.py | grep fold; done
done
