# Round 3: kernel trace of one C3 batch (both scorings) to see each query's
# fp16 launch, its rescue tail and the gaps between queries.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03c3trace}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-verify > $O/c3.json 2> $O/c3.err
rc=$?; echo RC=$rc; f=$(find $O/kt -name "*kernel_trace.csv"); ls -la $f; gzip -k $f; exit $rc
