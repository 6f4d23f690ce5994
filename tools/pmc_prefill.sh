#!/bin/bash
# Two PMC passes (counters only, no trace domains) over one prefill configuration.
set -u
OUT=${1:-gpurun_out/pmc_prefill}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
ARGS=${PMC_ARGS:-"1 8192 32 8"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"
rc=0
for i in 1 2; do
  eval C=\$P$i
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/prof_one_kernel.py run prefill $ARGS > "$OUT/p$i.log" 2>&1 || { rc=$?; break; }
  python3 tools/prof_one_kernel.py sum "$OUT/p$i" attn_prefill
done
exit $rc
