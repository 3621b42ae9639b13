#!/bin/bash
# PMC passes over tools/rc4_bench (one counter group per run).  Usage on the box: tools/rc4_prof.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-a}
OUT=$R/gpurun_out/rc4prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $OUT/p1 -o p1 --output-format csv -- $R/tools/rc4_bench 16384 1 > $OUT/p1.txt
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p2 -o p2 --output-format csv -- $R/tools/rc4_bench 16384 1 > $OUT/p2.txt
find $OUT -name "*counter_collection.csv"
