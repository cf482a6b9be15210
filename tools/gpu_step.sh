set -e
for i in 1 2 3; do
for v in old new; do BCNF_AMD_LIB=build_exp/lib$v.so timeout -k 10 120 python tools/abk.py; done
done
