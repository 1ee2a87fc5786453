// sw_intra_x2.hip — the two-subjects-per-wave intra-sequence kernel
// (the long-subject path; config C5).  Its body and
// the description of the method are in sw_intra_x2.h.
#include "sw_intra_x2.h"

#include <cstdlib>

namespace swk {

// The LDS conveyor (ix2 CONV: 1 KB per wave) wherever it leaves the
// occupancy as it is: every shape but RI 16, whose 53 KB image leaves no room
// for it at 3 workgroups per CU.
template <int RI, bool F16, bool LIST, bool LIN>
__global__ __launch_bounds__(kWavesPerWG * kLanes) void sw_intra_x2(IntraArgs a) {
    __shared__ typename ix2::IntraImg<RI, F16>::Elem img[ix2::img_elems<RI, F16>()];
    constexpr bool kConv = RI != 16;
    ix2::intra_x2_wg<RI, F16, LIST, LIN, true, false, kConv>(a, blockIdx.x, img);
}

int intra_x2_rows_for(int qlen, int longest, int wide, int forced) {
    // chunks x steps x (cell pairs per lane-step + conveyor/hand-off overhead)
    if (forced > 0) {  // sw_opts intra_x2_rows (tests: force a shape)
        const int ri = forced;
        if (ri == 4 || ri == 6 || ri == 8 || ri == 10 || ri == 12 || ri == 16) return ri;
        if (ri == kIntraX2MaxRI && wide >= 1) return ri;
    }
    int best_ri = 16;
    double best_cost = 1e300;
    for (int ri : {4, 6, 8, 10, 12, 16, kIntraX2MaxRI}) {
        if (ri == kIntraX2MaxRI && wide < 2) continue;
        const int chunk = kLanes * ri;
        const int nch = (qlen + chunk - 1) / chunk;
        // SIMD cycles per lane-step: ri rows x 6.8 ops x 4.25 + ~80 of conveyor
        const double cost = static_cast<double>(nch) * (longest + kLanes - 1) * (ri * 28.8 + 80.0);
        if (cost < best_cost) {
            best_cost = cost;
            best_ri = ri;
        }
    }
    return best_ri;
}

template <bool F16, bool LIST, bool LIN>
static hipError_t launch_intra_x2_t(const IntraArgs& a, int ri, hipStream_t s) {
    const int npairs = (a.nsubj + 1) / 2;
    const dim3 grid((npairs + kWavesPerWG - 1) / kWavesPerWG), block(kWavesPerWG * kLanes);
    switch (ri) {
        case 4: hipLaunchKernelGGL((sw_intra_x2<4, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case 6: hipLaunchKernelGGL((sw_intra_x2<6, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL((sw_intra_x2<8, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case 10: hipLaunchKernelGGL((sw_intra_x2<10, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case 12: hipLaunchKernelGGL((sw_intra_x2<12, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case 16: hipLaunchKernelGGL((sw_intra_x2<16, F16, LIST, LIN>), grid, block, 0, s, a); break;
        case kIntraX2MaxRI: hipLaunchKernelGGL((sw_intra_x2<kIntraX2MaxRI, F16, LIST, LIN>), grid, block, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Linear gaps (open == extend) take the biased linear cell (ix2 LIN), as in
// the merged launch (sw_scan_lpt); measured against the Farrar form in
// profiles/r02_intra_lin/.
bool intra_linear(const IntraArgs& a) { return a.gap_open == a.gap_extend; }

template <bool F16, bool LIST>
static hipError_t launch_intra_x2_g(const IntraArgs& a, int ri, hipStream_t s) {
    return intra_linear(a) ? launch_intra_x2_t<F16, LIST, true>(a, ri, s) : launch_intra_x2_t<F16, LIST, false>(a, ri, s);
}

hipError_t launch_intra_x2(const IntraArgs& a, int ri, hipStream_t s) {
    if (a.nsubj <= 0 || a.qpad <= 0) return hipSuccess;
    return launch_intra_x2_g<true, false>(a, ri, s);
}

// The int16 form over the device-side list of subjects the fp16 pass flagged
// (a.subj_list / a.list_count); it flags its own near-32767 subjects into
// a.rescue_list for the int32 sw_intra.
hipError_t launch_intra_x2_list16(const IntraArgs& a, int ri, hipStream_t s) {
    if (a.nsubj <= 0 || a.qpad <= 0) return hipSuccess;
    return launch_intra_x2_g<false, true>(a, ri, s);
}

hipError_t launch_intra_x2_int16(const IntraArgs& a, int ri, hipStream_t s) {
    if (a.nsubj <= 0 || a.qpad <= 0) return hipSuccess;
    return launch_intra_x2_g<false, false>(a, ri, s);
}

}  // namespace swk
