# Round 2: 26-code images and 3 ring slots (LDS of a quad workgroup 61 -> 48
# KB: 3 workgroups per CU): GPU suite, share of 8, C2, C3, with a short kernel
# trace of the share (LDS and VGPRs per kernel).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02w}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-verify"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 $B --shard-of 8 > $O/s8.json 2> $O/s8.err && \
timeout -k 10 300 $B > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 $B --config c3 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring --shard-of 8 --steps 10 > $O/kt.json 2> $O/kt.err
rc=$?; echo RC=$rc; tail -3 $O/pytest.log; for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('value_reference_scoring'), d.get('kernel_ms_per_scan'))"; done; exit $rc
