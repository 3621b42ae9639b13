#!/bin/bash
# round 5 session K: where an RC4 chain's time goes at 1 vs 9 waves per CU -- the chain-latency probe
# (tools/rc4_ksa_probe.hip time) under one rocprofv3 PMC pass: SQ_WAVE_CYCLES, SQ_WAIT_ANY (parked on s_waitcnt),
# SQ_WAIT_INST_ANY (ready, not issued), SQ_ACTIVE_INST_VALU / _LDS, SQ_INSTS_VALU / _LDS, GRBM_GUI_ACTIVE per dispatch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/pmc -o p --output-format csv -- $R/build/probe/probe_default time 2000 > $O/probe_time.jsonl 2>&1
echo "rc=$?" > $O/summary.txt
