// Host entry points of the specialised conv engines, each in its own translation unit so the
// big template files do not have to be rebuilt together.  Called from conv3d.hip's dispatch.
#pragma once
#include "common.h"

namespace vq3d {

// 1x1x1 weight gradient (and the epilogue-parameter gradients of that conv), ACCUMULATED:
//   G[co][ci] = sum_v g[v][co] * pro(x|x2)[v][ci]
//   dw += escale * G ; dscale += sum W*G ; dbias += sum g ; dcbias[co] += sum_v g[v][co]
// Partials per workgroup go to `workspace` (pw_wgrad_workspace(d) bytes) and are summed in a
// fixed order by a second kernel: deterministic, no same-address atomics.
size_t pw_wgrad_workspace(const vq3d_conv_desc *d);
int launch_pw_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pro_a,
                    const float *pro_b, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                    float *dcbias, void *workspace, size_t ws_bytes, hipStream_t s);

}  // namespace vq3d
