# Instruction-mix and MFMA-busy counters of the step kernel (via gpurun):
# how busy is the matrix pipe, and what do the element-wise phases issue?
# Two --pmc passes (<= 8 SQ + 2 GRBM counters each), each its own run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmc_sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/b1.json 2> $O/p1.err
echo P1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/b2.json 2> $O/p2.err

# vector-memory wavefronts by path: flat (scratch spills; no global/flat
# accesses in the N<=1024 step kernel besides them) vs buffer (records, alpha)
timeout -s KILL 120 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE \
    --output-format csv -d $O/p3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/b3.json 2> $O/p3.err
echo P3
timeout -s KILL 120 rocprofv3 --pmc TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE \
    --output-format csv -d $O/p4 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/b4.json 2> $O/p4.err
echo P4
echo DONE
