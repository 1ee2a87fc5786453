# Round 4: quads on/off (and a higher quad width) on the 1/2, 1/4, 1/8 shares and C3 (scripts/gpu_r04_sweep.sh per config)
set -o pipefail
RUN=r04sweep_s2 CFG="--shard-of 2" SWEEP="base:X=1 q0:SW_QUAD_WIDTH=0 q1800:SW_QUAD_WIDTH=1800" bash scripts/gpu_r04_sweep.sh && \
RUN=r04sweep_s4 CFG="--shard-of 4" SWEEP="base:X=1 q0:SW_QUAD_WIDTH=0 q1800:SW_QUAD_WIDTH=1800" bash scripts/gpu_r04_sweep.sh && \
RUN=r04sweep_s8 CFG="--shard-of 8" SWEEP="base:X=1 q0:SW_QUAD_WIDTH=0" bash scripts/gpu_r04_sweep.sh && \
RUN=r04sweep_c3 CFG="--config c3" SWEEP="base:X=1 q0:SW_QUAD_WIDTH=0" bash scripts/gpu_r04_sweep.sh
