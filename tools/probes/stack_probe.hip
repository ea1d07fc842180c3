// Phase clocks of the top-level stack chains (k_stackr_fwd / k_stackr_bwd): builds preact_stack.hip
// with VQ3D_STACK_PROBE, runs the published top level's run (50 blocks, 32 channels, branch 16,
// 8 x 8 x 2 voxels) forward and split backward, and prints per-block cycles between the probe
// points (0 top, 1 before the barrier, 2 after it, 3 after the conv, 4 end of block).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I3d-vq-vae-2_amd/csrc -Iinclude \
//         tools/probes/stack_probe.hip -o tools/probes/stack_probe && tools/probes/stack_probe
#define VQ3D_STACK_PROBE 1
#include "../../3d-vq-vae-2_amd/csrc/preact_stack.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

int vq3d_rt::fail(const std::string &msg) {
    fprintf(stderr, "fail: %s\n", msg.c_str());
    return 1;
}
int vq3d_rt::check_launch(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        return 1;
    }
    return 0;
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const int nb = 50, C = 32, B = 16, H = 8, W = 8, D = 2, nv = H * W * D;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    const int sizes[NPRM] = {B * C, B * B * 27, C * B, 1, 1, 1, 1, 1, 1, 1, 1};
    const float scl[NPRM] = {0.18f, 0.05f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 0.1f, 1.f, 0.1f};
    std::vector<float *> tab(nb * NPRM), gtab(nb * NPRM);
    for (int b = 0; b < nb; ++b)
        for (int k = 0; k < NPRM; ++k) {
            std::vector<float> h(sizes[k]);
            for (auto &v : h) v = k == 9 ? 1.f + 0.1f * nd(rng) : scl[k] * nd(rng);
            CK(hipMalloc(&tab[b * NPRM + k], sizes[k] * 4));
            CK(hipMemcpy(tab[b * NPRM + k], h.data(), sizes[k] * 4, hipMemcpyHostToDevice));
            CK(hipMalloc(&gtab[b * NPRM + k], sizes[k] * 4));
            CK(hipMemset(gtab[b * NPRM + k], 0, sizes[k] * 4));
        }
    float **dtab, **dgtab;
    CK(hipMalloc(&dtab, tab.size() * 8));
    CK(hipMalloc(&dgtab, gtab.size() * 8));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dgtab, gtab.data(), gtab.size() * 8, hipMemcpyHostToDevice));
    std::vector<uint16_t> hx(nv * C);
    for (auto &v : hx) {
        const float f = nd(rng);
        uint32_t u;
        std::memcpy(&u, &f, 4);
        v = uint16_t(u >> 16);
    }
    void *x, *out, *gx, *ws;
    float *saved;
    CK(hipMalloc(&x, nv * C * 2));
    CK(hipMalloc(&out, nv * C * 2));
    CK(hipMalloc(&gx, nv * C * 2));
    CK(hipMemcpy(x, hx.data(), nv * C * 2, hipMemcpyHostToDevice));
    const size_t ns = vq3d_preact_stack_saved_floats(nb, 1, C, B, H, W, D);
    CK(hipMalloc(&saved, ns * 4));
    const size_t nws = vq3d_preact_stack_bwd_workspace_bytes(nb, 1, C, B, H, W, D);
    CK(hipMalloc(&ws, nws));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const int reps = 20;
    float tf = 0.f, tb = 0.f;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(e0, 0));
        if (vq3d_preact_stack_fwd(VQ3D_HALF, nb, 1, C, B, H, W, D, x, dtab, out, saved, nullptr)) return 1;
        CK(hipEventRecord(e1, 0));
        if (vq3d_preact_stack_bwd_ws(VQ3D_HALF, nb, 1, C, B, H, W, D, out, dtab, dgtab, saved, gx, ws, nws, nullptr))
            return 1;
        CK(hipEventRecord(e2, 0));
        CK(hipEventSynchronize(e2));
        float a, b;
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventElapsedTime(&b, e1, e2));
        if (r >= 2) {
            tf += a;
            tb += b;
        }
    }
    printf("fwd (pack + chain) %.1f us, bwd (pack + chain + wgrad) %.1f us per run (events)\n", 1e3f * tf / reps,
           1e3f * tb / reps);
    unsigned long long pr[2][64][5];
    CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_stack_probe), sizeof(pr)));
    const char *name[2] = {"fwd", "bwd"};
    for (int d = 0; d < 2; ++d) {
        // per phase: median over blocks 3 .. 46 of stamp[k + 1] - stamp[k], and block-to-block
        std::vector<long long> ph[5];
        for (int b = 3; b < nb - 3; ++b) {
            for (int k = 0; k < 4; ++k) ph[k].push_back((long long)(pr[d][b][k + 1] - pr[d][b][k]));
            const int nxt = d == 0 ? b + 1 : b - 1;
            ph[4].push_back((long long)(pr[d][nxt][0] - pr[d][b][0]));
        }
        printf("%s medians (s_memtime ticks):", name[d]);
        const char *lab[5] = {"top->prebar", "barrier", "conv", "tail", "block"};
        for (int k = 0; k < 5; ++k) {
            std::sort(ph[k].begin(), ph[k].end());
            printf("  %s %lld", lab[k], ph[k][ph[k].size() / 2]);
        }
        printf("  | whole chain %llu ticks\n", d == 0 ? pr[d][nb - 1][4] - pr[d][0][0] : pr[d][0][4] - pr[d][nb - 1][0]);
    }
    return 0;
}
