# Round 2: host enqueue time per step vs GPU time (is the 1/8 share's step
# overhead host-bound?), with a kernel trace of the share.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02q}
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --shard-of 8 --no-overlap > $O/s8_serial.json 2> $O/s8_serial.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --shard-of 8 --steps 30 > $O/kt.json 2> $O/kt.err
rc=$?; echo RC=$rc; grep "host enqueue" $O/s8.err $O/s8_serial.err; ls $O/kt; exit $rc
