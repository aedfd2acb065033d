// siren_params.h — layout of the flat parameter buffer (nn.Linear / state_dict order, include/siren_amd.h).
#pragma once
#include "siren_common.h"

namespace siren {

// ------------------------------------------------------------------------------------------------------
// Parameter offsets inside the flat buffer (nn.Linear / state_dict order, see include/siren_amd.h).
// ------------------------------------------------------------------------------------------------------
struct ParamOffsets {
    int64_t w0, b0, hidden0, wout, bout, total, h;
    __host__ __device__ ParamOffsets(int d, int o, int lh, int hw = H) {
        h = hw;
        w0 = 0;
        b0 = h * d;
        hidden0 = b0 + h;
        wout = hidden0 + (int64_t)lh * (h * h + h);
        bout = wout + (int64_t)o * h;
        total = bout + o;
    }
    __host__ __device__ int64_t w(int l) const { return hidden0 + (int64_t)(l - 1) * (h * h + h); }
    __host__ __device__ int64_t b(int l) const { return l == 0 ? b0 : w(l) + h * h; }
};


}  // namespace siren
