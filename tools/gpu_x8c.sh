#!/bin/bash
# GPU: the 8-window chained step in several layouts (tools/x8_chain_split.py; LAYOUTS="K ovl mode ...")
set -e
mkdir -p gpurun_out
L=gpurun_out/x8c_layouts.log
for a in ${LAYOUTS:-"4 0 group" "3 0 group" "4 1 group" "8 0 solo"}; do
  timeout -k 10 100 python -u tools/x8_chain_split.py $a >> $L 2>&1
done
