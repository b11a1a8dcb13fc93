#!/bin/bash
# Cluster-size sweep of the clustered leaf scan on c3 (ATR_CLUSTER_SIZE read at scene upload).
export TMPDIR=/tmp
mkdir -p gpurun_out/clsweep
for S in ${SIZES:-4 8 12 16 24 32}; do
  ATR_CLUSTER_SIZE=$S timeout -k 10 200 python tools/kprof.py --config ${CONFIG:-c3} --variants ${VARS:-cl} --rounds 3 --iters 5 > gpurun_out/clsweep/s$S.json 2> gpurun_out/clsweep/s$S.err
  rc=$?; echo "size $S rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
