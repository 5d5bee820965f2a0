O=gpurun_out/r1s23; mkdir -p $O
for mode in off edge sa; do
  PCOPS_CONV1X1=$mode timeout -k 10 150 python bench.py --model pointsea --no-cpu-baseline --no-kernel-timing --steps 3 --warmup 2 > $O/ps_$mode.json 2> $O/ps_$mode.err; echo "$mode rc=$?"
done
