# GPU box: device times of the folded training pass with the pack-free forward on / off, plus the phase stamps of a
# diagnostic build (tools/exp_variants.sh stamps) and any experiment builds named in RAW_LIBS.
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 120 python tools/raw_probe.py
BCNF_FOLD_RAW=0 timeout -k 10 120 python tools/raw_probe.py
for lib in $RAW_LIBS; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/raw_probe.py; done
done
BCNF_AMD_LIB=build_exp/libstamps.so timeout -k 10 120 python tools/raw_probe.py
BCNF_FOLD_RAW=0 BCNF_AMD_LIB=build_exp/libstamps.so timeout -k 10 120 python tools/raw_probe.py
