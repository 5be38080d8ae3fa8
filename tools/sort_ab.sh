B="python bench.py --no-encode --no-cpu-baseline"
for r in 1 2; do
 for l in ab/libbpe_head.so ab/libbpe_alt.so ab/libbpe_s256.so; do
  n=$(basename $l .so)
  BPE_LIB=$l timeout -k 10 200 $B > gpurun_out/st_${n}_$r.json 2>/dev/null || exit 1
 done
done
echo done
