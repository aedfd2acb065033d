// siren_params.h — layout of the flat parameter buffer (nn.Linear / state_dict order, include/siren_amd.h).
#pragma once
#include "siren_common.h"

namespace siren {

// ------------------------------------------------------------------------------------------------------
// Parameter offsets inside the flat buffer (nn.Linear / state_dict order, see include/siren_amd.h).
// ------------------------------------------------------------------------------------------------------
struct ParamOffsets {
    int64_t w0, b0, hidden0, wout, bout, total;
    __host__ __device__ ParamOffsets(int d, int o, int lh) {
        w0 = 0;
        b0 = (int64_t)H * d;
        hidden0 = b0 + H;
        wout = hidden0 + (int64_t)lh * (H * H + H);
        bout = wout + (int64_t)o * H;
        total = bout + o;
    }
    __host__ __device__ int64_t w(int l) const { return hidden0 + (int64_t)(l - 1) * (H * H + H); }
    __host__ __device__ int64_t b(int l) const { return l == 0 ? b0 : w(l) + (int64_t)H * H; }
};


}  // namespace siren
