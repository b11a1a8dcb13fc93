#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/balsweep
for S in ${BS_STREAMS:-2 4 6 8}; do
  timeout -k 10 300 python tools/shard_balance.py --plans lpt --sides ${BS_SIDES:-32,64} --worlds ${BS_WORLDS:-2,4,8} --streams $S --iters 6 > gpurun_out/balsweep/s$S.json 2> gpurun_out/balsweep/s$S.err
  rc=$?; echo "s$S rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done
