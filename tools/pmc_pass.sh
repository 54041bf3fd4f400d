#!/bin/bash
# SQ / SQC / TA counter passes (separate --pmc runs, no tracing) of a short
# bench run: bash tools/pmc_pass.sh <outdir>.  At most 2 TA counters per pass
# (rocprofv3 does not split passes; 3 TA counters hang it): the record
# traffic (TA_BUFFER_* -- MUBUF, the solver records and alpha), the FLAT-
# encoded traffic (TA_FLAT_* -- scratch spills / call frames plus the few
# global accesses), and TA busy each get a run of their own.
# A counter the device does not list is skipped (rocprofv3 -L first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
have() { grep -q -w "$1" $O/counters.txt; }
pass() {  # pass <name> <counters...>
    local name=$1; shift
    local use=()
    for c in "$@"; do have $c && use+=($c); done
    [ ${#use[@]} -eq 0 ] && { echo "skip $name (none listed)"; return 0; }
    echo "pass $name: ${use[*]}"
    timeout -s KILL 180 rocprofv3 --pmc ${use[*]} --output-format csv -d $O/$name -o run -- \
        python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/$name.json 2> $O/$name.err
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC &&
pass sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS &&
pass sqc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE &&
pass ta_buf TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum &&
pass ta_flat TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum &&
pass ta_busy TA_BUSY_avr TA_TA_BUSY_sum
echo "pmc rc=$?"
