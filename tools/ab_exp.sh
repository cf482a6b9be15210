# A/B of experiment builds (GPU box): bash tools/ab_exp.sh 1 8 2048 ...  (default library first)
set -e
timeout -k 10 120 python tools/abk.py
for e in "$@"; do BCNF_AMD_LIB=build_exp/libexp$e.so timeout -k 10 120 python tools/abk.py; done
