# Round 3 A/B on one box: the library variants in $LIBS (dirs under the
# package; "lib" = the default build) on the configs in $CONFIGS, alternated
# twice; then, with TRACE=1, raw block timelines of C2's 1/8 share and the
# whole C2 from the -DSW_TRACE_BLOCKS build (lib_trace).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r03ab}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
b() { tag=$1; lib=$2; shift 2; SW_AMD_LIB=$P/$lib/libswamd.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-verify "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAILED"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]); r=d.get('reference_scoring',{})
print('$tag', d['value'], d['ms_per_step'], d.get('kernel_ms_per_scan',{}).get('scan_total'), r.get('value'), r.get('ms_per_step'))"; }
for rep in 1 2; do
  for lib in ${LIBS:-lib}; do
    for c in ${CONFIGS:-s8}; do
      case $c in
        c2) b ${c}_${lib}_$rep $lib ;;
        s8) b ${c}_${lib}_$rep $lib --shard-of 8 ;;
        s4) b ${c}_${lib}_$rep $lib --shard-of 4 ;;
        c3) b ${c}_${lib}_$rep $lib --config c3 ;;
        c5) b ${c}_${lib}_$rep $lib --config c5 ;;
      esac
    done
  done
done
if [ -n "$TRACE" ]; then
  for s in 8 1; do
    SW_AMD_LIB=$P/lib_trace/libswamd.so SW_TRACE_FILE=/tmp/sw_trace_$s.bin timeout -k 10 300 python3 scripts/exp_share_dump.py $s $O/trace_s$s.npz > $O/trace_s$s.log 2>&1 || { echo TRACE FAILED; tail $O/trace_s$s.log; exit 1; }
  done
  echo traces ok
fi
