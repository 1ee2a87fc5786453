# Round 6: block / workgroup timelines (the -DSW_TRACE_BLOCKS build,
# lib_trace) of rank $SRANK's share of C2 at N = $SHARD under both scorings,
# as .npz dumps for scripts/trace_occupancy.py and offline analysis.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06trace}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
for sc in aff ref; do
  a=""; [ $sc = ref ] && a="0 ref"
  SW_AMD_LIB=$P/lib_trace/libswamd.so SW_TRACE_FILE=/tmp/sw_trace_$sc.bin timeout -k 10 300 \
    python3 scripts/exp_share_dump.py ${SHARD:-8}:${SRANK:-0} $O/s${SHARD:-8}_r${SRANK:-0}_$sc.npz $a > $O/dump_$sc.log 2>&1 \
    || { echo "TRACE $sc FAILED"; tail $O/dump_$sc.log; exit 1; }
  python3 scripts/trace_occupancy.py $O/s${SHARD:-8}_r${SRANK:-0}_$sc.npz
done
echo RC=0
