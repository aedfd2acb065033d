// tu_legacy.hip — pack kernel and the round-1 fused kernels (runtime layer loop; notebook final-sine nets,
// forward-only depths 6..8, and the SIREN_FLAG_LEGACY_KERNEL A/B reference).
#include "fused_kernels.hpp"
#include "launch.h"

namespace siren {

void launch_pack(const float* p, float* ws, int d, int o, int lh, int h, int64_t spad, int64_t total, int64_t base,
                 float s0, float s, hipStream_t st, int batch, int64_t p_bstride, int64_t begin) {
    const int threads = 256;
    const int64_t blocks = std::min<int64_t>(((total - begin) / 4 + threads - 1) / threads, 8192);  // one quad / thread
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1), (unsigned)batch), dim3(threads), 0,
                       st, p, ws, d, o, lh, spad, total, h, base, s0, s, p_bstride, begin);
}

void launch_legacy_fwd(dim3 grid, hipStream_t st, const FusedArgs& a) {
    hipLaunchKernelGGL((fused_kernel<0, false>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, nullptr, a.y, nullptr,
                       a.d, a.o, a.lh, a.w0, a.w, a.final_sine, nullptr, nullptr, (int64_t)0);
}

void launch_legacy_grad(bool store, dim3 grid, hipStream_t st, const FusedArgs& a) {
#define SIREN_L(LHV, ST)                                                                                    \
    hipLaunchKernelGGL((fused_kernel<LHV, true, ST>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx, \
                       a.d, a.o, LHV, a.w0, a.w, a.final_sine, a.abuf, a.dbuf, a.n_pad)
    if (store) {
        switch (a.lh) {
            case 1: SIREN_L(1, true); break;
            case 2: SIREN_L(2, true); break;
            default: SIREN_L(3, true); break;
        }
    } else {
        switch (a.lh) {
            case 1: SIREN_L(1, false); break;
            case 2: SIREN_L(2, false); break;
            default: SIREN_L(3, false); break;
        }
    }
#undef SIREN_L
}

}  // namespace siren
