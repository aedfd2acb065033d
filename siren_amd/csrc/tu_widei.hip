// tu_widei.hip — dispatch of the hidden-512 stored-forward split with interleaved epilogues (widei_kernel.hpp); the
// instantiations live in tu_widei_{fa,fb,ra,rb}.hip (compile-time partitioning: each LH is a fully unrolled kernel).
#include "launch.h"
#include "siren_common.h"

namespace siren {

void launch_widei_fa(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);
void launch_widei_fb(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);
void launch_widei_ra(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);
void launch_widei_rb(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill);

bool launch_widei(int mode, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill) {
    if (a.lh < 1 || a.lh > 5 || a.final_sine != 0 || (mode != MODE_FWDS && mode != MODE_REV)) return false;
    if (mode == MODE_FWDS)
        (a.lh <= 3 ? launch_widei_fa : launch_widei_fb)(a.lh, grid, st, a, spill);
    else
        (a.lh <= 3 ? launch_widei_ra : launch_widei_rb)(a.lh, grid, st, a, spill);
    return true;
}

}  // namespace siren
