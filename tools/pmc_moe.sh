#!/bin/bash
# PMC passes (counters only, no trace domains) over the Mixtral w13+SwiGLU grouped GEMM.
set -u
OUT=${1:-gpurun_out/pmc_moe}; shift || true
T=${PMC_T:-3072}
TILE=${PMC_TILE:-256}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P2="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUFFER_WAVEFRONTS_sum"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
rc=0
for i in 1 2 3; do
  eval C=\$P$i
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/prof_one_kernel.py run moe $T $TILE > "$OUT/p$i.log" 2>&1 || { rc=$?; echo "pass $i rc=$rc"; tail -3 "$OUT/p$i.log"; continue; }
  python3 tools/prof_one_kernel.py sum "$OUT/p$i" moe_gemm
done
exit $rc
