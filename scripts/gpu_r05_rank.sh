# Round 5, VERDICT r04 item 4: the device top-K in one launch
# (sw_topk_fused) on the exchange stream beside the next scan.  The GPU
# tests of every ranking path, then C2 and its 1/8 share with the one-launch
# top-K against the chained stages (lib_chain: -DSW_TOPK_FUSED=0),
# alternated $REPS times, then kernel traces of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05rank}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rank.py \
    tests/test_gpu_overlap.py tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_device_topk" \
    "tests/test_gpu_parity.py::test_device_topk_radix_select" tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
B="bench.py --no-cpu-baseline --no-verify --sustained-seconds 0"
for rep in $(seq 1 ${REPS:-2}); do
  for form in fused chain; do
    lib=$P/lib/libswamd.so; [ $form = chain ] && lib=$P/lib_chain/libswamd.so
    for c in ${CFGS:-c2 s8}; do
      case $c in s8) a="--shard-of 8" ;; c2) a="" ;; esac
      SW_AMD_LIB=$lib timeout -k 10 300 python3 $B $a > $O/${c}_${form}_$rep.json 2> $O/${c}_${form}_$rep.err || { echo "$c $form FAILED"; tail -20 $O/${c}_${form}_$rep.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/${c}_${form}_$rep.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$c $form $rep', d['value'], d['ms_per_step'], r.get('value'), r.get('ms_per_step'), d['kernels']['inter'])"
    done
  done
done
for form in fused chain; do
  lib=$P/lib/libswamd.so; [ $form = chain ] && lib=$P/lib_chain/libswamd.so
  for c in ${CFGS:-c2 s8}; do
    case $c in s8) a="--shard-of 8" ;; c2) a="" ;; esac
    SW_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${c}_$form -o run --output-format csv -- python3 $B $a --no-reference-scoring --steps 20 > $O/kt_${c}_$form.json 2> $O/kt_${c}_$form.err || { echo "TRACE $c $form FAILED"; tail -5 $O/kt_${c}_$form.err; exit 1; }
    cp $(find $O/kt_${c}_$form -name "*kernel_stats.csv") $O/${c}_${form}_kernel_stats.csv
    python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(sys.argv[2], r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])" $O/${c}_${form}_kernel_stats.csv ${c}_$form
  done
done
echo RC=0
