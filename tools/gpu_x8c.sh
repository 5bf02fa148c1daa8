set -e
mkdir -p gpurun_out
L=gpurun_out/x8c2.log
for a in "8 0 solo" "8 0 group" "4 0 group" "2 0 group" "1 0 group" "4 1 group" "8 1 solo"; do
  timeout -k 10 100 python -u tools/x8_chain_split.py $a >> $L 2>&1
done
