# Round 3 A/B: wave priority for the merged launch's longest workgroups
# (SW_LPT_PRIO = fraction of the longest estimated duration), with the
# paired inter steps (lib) and without (lib_base, -DSW_X2_PAIR=0), on C2's
# 1/8 and 1/4 shares
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-s3p}; mkdir -p $O
LB=ece1782-smith-waterman-cuda_amd/lib_base/libswamd.so
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "lpt or merged or share or group or pair or quad" > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify --no-reference-scoring $ARGS > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1])
print('$tag', d['value'], d['ms_per_step'])"; }
for n in 8 4; do ARGS="--shard-of $n"
  for rep in 1 2; do
    run s${n}_pair_p0_$rep X=1
    run s${n}_base_p0_$rep SW_AMD_LIB=$LB
    for pf in 0.9 0.7 0.5; do
      run s${n}_pair_p${pf}_$rep SW_LPT_PRIO=$pf
      run s${n}_base_p${pf}_$rep SW_LPT_PRIO=$pf SW_AMD_LIB=$LB
    done
  done
done
