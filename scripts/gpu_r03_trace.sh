# Round 3: kernel + copy trace of C2's 1/8 share (gaps between a step's
# launches), the C3 and C5 lines, a kernel trace of one C3 batch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/s8 -o run --output-format csv -- python3 bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $O/s8.json 2> $O/s8.err || { echo S8 TRACE FAILED; tail -20 $O/s8.err; exit 1; }
for f in $(find $O/s8 -name "*.csv"); do gzip $f; done
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }; }
b c3 --config c3
b c5 --config c5
RUN=r03trace/c3trace bash scripts/gpu_r03_c3trace.sh
for f in c3 c5; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$f', d['value'], d['ms_per_step'], d.get('kernels'), r.get('value'), r.get('ms_per_step'), d.get('parity_sample_ok'))"; done
