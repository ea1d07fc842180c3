// Phase clocks of the brick backward k_small_bwd<8,4,float,float> at the published pre-quantize
// level (8 channels, branch 4, 32 x 32 x 8 voxels, 128 bricks): builds preact_small.hip with
// SMALL_PROBE and prints, over the workgroups, the median s_memtime ticks between the probe points
// (0 start, 1 weight-staging barrier, 2 phase 1 barrier, 3 phase 2 done, 4 W2 sub-stream barrier,
// 5 partial rows + wave sums barrier, 6 end; inside phase 2 / 3: taps, tap barrier, sum +
// epilogue, per-thread sums to LDS, W2 gradient).  Sched barriers keep code on its side of a probe.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -c tools/probes/small_probe.hip -o /tmp/sp.o && \
//   hipcc --offload-arch=gfx950 /tmp/sp.o 3d-vq-vae-2_amd/build/preact_col.o -o tools/probes/small_probe
#define SMALL_PROBE 1
#include "../../3d-vq-vae-2_amd/csrc/preact_small.hip"

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

static int upload(std::vector<float> &h, float **d) {
    CK(hipMalloc(d, h.size() * 4));
    CK(hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return 0;
}

int main() {
    const int C = 8, B = 4, H = 32, W = 32, D = 8, nv = H * W * D;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    auto randv = [&](size_t n, float s) {
        std::vector<float> v(n);
        for (auto &e : v) e = s * nd(rng);
        return v;
    };
    std::vector<float> hx = randv(size_t(nv) * C, 1.f), hg = randv(size_t(nv) * C, 1.f);
    std::vector<float> hw1 = randv(B * C, 0.3f), hw2 = randv(27 * B * B, 0.1f), hw3 = randv(C * B, 0.3f);
    std::vector<uint16_t> ht(size_t(nv) * B);
    for (auto &v : ht) {
        const float f = nd(rng);
        uint32_t u;
        std::memcpy(&u, &f, 4);
        v = uint16_t(u >> 16);
    }
    float *x, *g, *w1, *w2, *w3, *gx, *sc[8], *gr[11];
    if (upload(hx, &x) || upload(hg, &g) || upload(hw1, &w1) || upload(hw2, &w2) || upload(hw3, &w3)) return 1;
    for (int i = 0; i < 8; ++i) {
        std::vector<float> v(1, i == 6 ? 1.f : 0.1f);
        if (upload(v, &sc[i])) return 1;
    }
    const int gsz[11] = {B * C, 27 * B * B, C * B, 1, 1, 1, 1, 1, 1, 1, 1};
    for (int i = 0; i < 11; ++i) {
        std::vector<float> v(gsz[i], 0.f);
        if (upload(v, &gr[i])) return 1;
    }
    void *t2, *t3, *ws;
    CK(hipMalloc(&t2, ht.size() * 2));
    CK(hipMalloc(&t3, ht.size() * 2));
    CK(hipMemcpy(t2, ht.data(), ht.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(t3, ht.data(), ht.size() * 2, hipMemcpyHostToDevice));
    CK(hipMalloc(&gx, size_t(nv) * C * 4));
    const size_t nws = vq3d_preact_small_workspace_bytes(1, C, B, H, W, D);
    CK(hipMalloc(&ws, nws));
    const vq3d_preact_params p{sc[0], sc[1], sc[2], sc[3], sc[4], sc[5], sc[6], sc[7]};
    const vq3d_preact_grads G{gr[0], gr[1], gr[2], gr[3], gr[4], gr[5], gr[6], gr[7], gr[8], gr[9], gr[10]};
    SArgs a;
    if (!plan(1, C, B, H, W, D, a)) return 1;
    const int nb = std::min(a.nbricks, 1024);
    const int reps = 20;
    std::vector<long long> ph[7], sub[5], whole;
    for (int r = 0; r < reps + 2; ++r) {
        if (vq3d_preact_small_bwd_stages_io(1, VQ3D_HALF, VQ3D_F32, VQ3D_F32, 1, C, B, H, W, D, g, x, t2, t3, w1, w2, w3,
                                            &p, &G, ws, nws, gx, nullptr))
            return 1;
        CK(hipDeviceSynchronize());
        if (r < 2) continue;
        static unsigned long long pr[1024][12];
        CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_small_probe), sizeof(pr)));
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int b = 0; b < nb; ++b) {
            for (int k = 0; k < 6; ++k) ph[k].push_back((long long)(pr[b][k + 1] - pr[b][k]));
            ph[6].push_back((long long)(pr[b][7] - pr[b][6]));
            const int chain[6] = {2, 8, 9, 3, 10, 4};  // phase 2 taps, tap barrier, sum + epilogue, rt writes, phase 3
            for (int k = 0; k < 5; ++k) sub[k].push_back((long long)(pr[b][chain[k + 1]] - pr[b][chain[k]]));
            t0 = std::min(t0, pr[b][0]);
            t1 = std::max(t1, pr[b][7]);
        }
        whole.push_back((long long)(t1 - t0));
    }
    printf("k_small_bwd<8,4,f32,f32> @32x32x8 (%d bricks of %d voxels, halo %d): medians over workgroups x %d runs, "
           "s_memtime ticks\n", a.nbricks, a.nvb, a.hp, reps);
    const char *lab[7] = {"staging", "phase1", "phase2", "w2grad", "rows+wavesums", "red2", "tail"};
    for (int k = 0; k < 7; ++k) {
        std::sort(ph[k].begin(), ph[k].end());
        printf("  %-14s %6lld  (p90 %lld)\n", lab[k], ph[k][ph[k].size() / 2], ph[k][ph[k].size() * 9 / 10]);
    }
    const char *sl[5] = {"taps", "tap barrier", "sum+epilogue", "sum rows->LDS", "phase 3"};
    for (int k = 0; k < 5; ++k) {
        std::sort(sub[k].begin(), sub[k].end());
        printf("    %-14s %6lld\n", sl[k], sub[k][sub[k].size() / 2]);
    }
    std::sort(whole.begin(), whole.end());
    return 0;
}
