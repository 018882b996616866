#!/bin/bash
# Sample GPU clock / power / temperature while the C2 bench loops (is the FP64 kernel power-limited?)
cd "$(dirname "$0")/.."
OUT=gpurun_out/clock; mkdir -p $OUT
timeout -k 10 120 python bench.py --steps ${STEPS:-400} --warmup 2 --no-cpu-baseline --no-host-path > $OUT/bench.json 2> $OUT/bench.err &
P=$!
sleep ${DELAY:-12}
for i in 1 2 3 4 5; do
  timeout 20 rocm-smi --showclocks --showpower --showtemp --showuse > $OUT/smi_$i.txt 2>&1
  sleep 1
done
wait $P
echo "bench rc=$?"; cat $OUT/bench.json | head -c 400; echo
grep -h -i "sclk\|power\|fclk\|mclk\|use\|edge\|junction" $OUT/smi_3.txt | head -20
