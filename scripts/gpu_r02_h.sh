# Round 2: timelines of the merged launch on the strong-scaling shares.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02h}
mkdir -p $O
L=ece1782-smith-waterman-cuda_amd/lib_trace/libswamd.so
for cfg in "8 0" "4 0" "8 512" "8 1024"; do
  set -- $cfg
  SW_AMD_LIB=$L SW_TRACE_FILE=/tmp/tr.bin timeout -k 10 200 python3 scripts/exp_share_trace.py $1 $2 > $O/lpt_s$1_t$2.json 2> $O/lpt_s$1_t$2.err || exit 1
done
echo RC=0; for f in $O/lpt_*.json; do echo $f; cat $f; echo; done
