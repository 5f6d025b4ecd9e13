#!/bin/bash
# A/B of engine variants on the GPU box: run_ab.sh "cfg1;cfg2;..." lib1.so lib2.so ...
# (each step under its own time limit; stops at the first failure)
set -euo pipefail
mkdir -p gpurun_out
log=gpurun_out/ab.log
: > $log
IFS=';' read -ra cfgs <<< "$1"
shift
for cfg in "${cfgs[@]}"; do
  echo "== $cfg" >> $log
  timeout -k 10 120 python microbench/ab.py "$@" $cfg >> $log 2>&1
done
cat $log
