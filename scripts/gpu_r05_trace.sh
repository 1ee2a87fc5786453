# Round 5: block / workgroup timelines of C2's 1/8 share from the
# -DSW_TRACE_BLOCKS build (lib_trace), under the reference scoring (BLOSUM50,
# linear 2) and the affine default, for the critical path of each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05trace}
mkdir -p $O
P=ece1782-smith-waterman-cuda_amd
for sc in ref aff; do
  SW_AMD_LIB=$P/lib_trace/libswamd.so SW_TRACE_FILE=/tmp/sw_trace_$sc.bin timeout -k 10 300 \
    python3 scripts/exp_share_trace.py ${SHARD:-8} 0 $sc > $O/trace_s8_$sc.json 2> $O/trace_s8_$sc.err \
    || { echo "TRACE $sc FAILED"; tail $O/trace_s8_$sc.err; exit 1; }
  cat $O/trace_s8_$sc.json
done
echo RC=0
