#!/bin/bash
# PMC passes over a probe (PROBE, default tools/pmc_probe.py; e.g. PROBE="tools/path_probe.py c4 0 1"),
# one counter group per rocprofv3 run (--kernel-trace only), each under its own time limit.
# Output: gpurun_out/$OUT_DIR/g<i>/..., summarized by tools/pmc_summary2.py.
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-pmc2}
mkdir -p $O
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/g$i -o p -- python3 ${PROBE:-tools/pmc_probe.py} > $O/g$i.log 2>&1
  rc=$?; echo "group $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum
TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH
TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum TCP_TCC_WRITE_REQ_sum
SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES
FETCH_SIZE
WRITE_SIZE
GROUPS
echo done
