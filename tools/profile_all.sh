#!/bin/bash
# Profile every bench workload (kernel-trace/stats + the PMC passes of profile_gpu.sh), one after the other;
# stops at the first failing step.  Usage on the box: tools/profile_all.sh <tag> [workloads...]
set -e
TAG=${1:-r02}; shift || true
WL=${@:-odt office odt_e pdf_r34 pdf_r3 pdf_r3_40 pdf_r6 pdf_r2 pdf_r5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
for W in $WL; do
  echo "== $W $(date +%T)"
  bash $R/tools/profile_gpu.sh $W $TAG > /dev/null
done
echo done
