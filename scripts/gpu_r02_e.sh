# Round 2: block timelines of the strong-scaling shares (trace build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r02e}
mkdir -p $O
L=ece1782-smith-waterman-cuda_amd/lib_trace/libswamd.so
for cfg in "8 704 2" "8 704 4" "8 2048 2" "4 1024 2" "1 0 2"; do
  set -- $cfg
  SW_PAIR_GROUP=$3 SW_AMD_LIB=$L SW_TRACE_FILE=/tmp/tr.bin timeout -k 10 200 python3 scripts/exp_share_trace.py $1 $2 > $O/trace_s$1_t$2_g$3.json 2> $O/trace_s$1_t$2_g$3.err || exit 1
done
echo RC=0; for f in $O/trace_*.json; do echo $f; cat $f; echo; done
