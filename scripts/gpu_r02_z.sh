# Round 2: bisect the C3 reference-scoring slowdown (12,941 -> 8,900 GCUPS)
# over earlier builds: for each commit C in $BISECT, first (on the CPU side)
#   git worktree add .bisect/C C && make -C .bisect/C/ece1782-smith-waterman-cuda_amd/csrc
# (.bisect/ is excluded from git; the built trees travel with gpurun).
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/${RUN:-r02z}
mkdir -p $O
for c in ${BISECT:-34c3cba eager}; do
  (cd .bisect/$c && timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline --no-verify > $O/c3_$c.json 2> $O/c3_$c.err) || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('reference_scoring') or {}; print('$f', d['value'], d['ms_per_step'], '| ref', r.get('value'), r.get('kernel'), r.get('intra_kernel'), r.get('kernel_ms_per_scan'))"; done
