set -e
timeout -k 10 120 python tools/abk.py
for e in 2 4 6 512 1024; do BCNF_AMD_LIB=build_exp/libexp$e.so timeout -k 10 120 python tools/abk.py; done
