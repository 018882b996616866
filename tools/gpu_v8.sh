set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/v8; mkdir -p $OUT
echo "== bench s2" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_s2.json 2> $OUT/bench_s2.err \
&& echo "== bench s1" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --streams 1 --no-cpu-baseline --no-host-path > $OUT/bench_s1.json 2> $OUT/bench_s1.err \
&& echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_prof.json 2> $OUT/prof.err
rc=$?
cat $OUT/bench_s2.json $OUT/bench_s1.json $OUT/bench_prof.json
python tools/trace_span.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1)
exit $rc
