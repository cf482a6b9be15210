set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== default"; timeout -k 10 120 python tools/kbench.py
# (r05: the BCNF_LDS_MIN_KB occupancy knob was removed from the library)
echo "== batch 1024"; timeout -k 10 120 python tools/kbench.py --batch 1024
echo "== batch 16384"; timeout -k 10 120 python tools/kbench.py --batch 16384
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc1 -o pmc1 -- python tools/kbench.py --iters 5 > gpurun_out/pmc1.log 2>&1
echo pmc_done
