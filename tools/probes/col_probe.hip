// Phase clocks of the column backward k_col_bwd<C,BR,float,float> (first brick of each workgroup)
// at the published shapes: (2, 1) @ 128x128x32, (4, 2) @ 512x512x128, (8, 4) @ 256x256x64.  Builds
// preact_col.hip with COL_PROBE; prints the median s_memtime ticks between the probe points
// (0 start, 1 line table, 2 phase A barrier, 3 phase B barrier, 4 phase C done, 5 partial sums
// put, 6 partial row written).  Sched barriers keep code on its side of a probe.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/probes/col_probe tools/probes/col_probe.hip
//   tools/probes/col_probe 2 [h|f] [c]  (C = 2, 4 or 8; "h": 16-bit x / g, else fp32; "c": cold caches
//   between launches; -DNO_COL_PROBE: no clocks)
#ifndef NO_COL_PROBE
#define COL_PROBE 1
#endif
#include "../../3d-vq-vae-2_amd/csrc/preact_col.hip"

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

int main(int argc, char **argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 2, B = C / 2;
    const int dt = argc > 2 && argv[2][0] == 'h' ? int(vq3d::VQ3D_HALF) : int(VQ3D_F32);  // x / g storage ("h": 16-bit)
    const bool cold = argc > 3 && argv[3][0] == 'c';  // "c": a 1 GiB memset between launches (cold L2 / MALL)
    void *flush = nullptr;
    if (cold) CK(hipMalloc(&flush, size_t(1) << 30));
    const int H = C == 2 ? 128 : C == 4 ? 512 : 256, W = H, D = C == 2 ? 32 : C == 4 ? 128 : 64;
    const size_t nv = size_t(H) * W * D;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    auto randv = [&](size_t n, float s) {
        std::vector<float> v(n);
        for (auto &e : v) e = s * nd(rng);
        return v;
    };
    std::vector<float> hx = randv(nv * C, 1.f), hg = randv(nv * C, 1.f);
    std::vector<float> hw1 = randv(B * C, 0.3f), hw2 = randv(27 * B * B, 0.1f), hw3 = randv(C * B, 0.3f);
    std::vector<uint16_t> ht(nv * B);
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
    CK(hipMalloc(&gx, nv * C * 4));
    const size_t nws = vq3d::col_workspace_bytes(1, C, B, H, W, D);
    CK(hipMalloc(&ws, nws));
    const vq3d_preact_params p{sc[0], sc[1], sc[2], sc[3], sc[4], sc[5], sc[6], sc[7]};
    const vq3d_preact_grads G{gr[0], gr[1], gr[2], gr[3], gr[4], gr[5], gr[6], gr[7], gr[8], gr[9], gr[10]};
    const vq3d::CArgs a = vq3d::make_args(1, H, W, D);
    const int nb = std::min(a.nwg, 4096);
    const int reps = 20;
    std::vector<long long> ph[6];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0.f;
    for (int r = 0; r < reps + 2; ++r) {
        if (cold) CK(hipMemsetAsync(flush, r & 0xff, size_t(1) << 30, 0));
        CK(hipEventRecord(e0, 0));
        if (vq3d::col_bwd(dt, dt, 1, C, B, H, W, D, g, x, t2, t3, w1, w2, w3, p, G, ws, gx, 1, nullptr))
            return 1;
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        if (r < 2) continue;
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms += t;
#ifndef NO_COL_PROBE
        static unsigned long long pr[4096][8];
        CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_col_probe), sizeof(pr)));
        for (int b = 0; b < nb; ++b)
            for (int k = 0; k < 6; ++k) ph[k].push_back((long long)(pr[b][k + 1] - pr[b][k]));
#else
        (void)nb;
#endif
    }
    printf("k_col_bwd<%d,%d,f32,f32> @%dx%dx%d (%d bricks, %d workgroups): %.1f us per launch (events); "
           "medians over workgroups x %d runs, s_memtime ticks\n", C, B, H, W, D, a.nbricks, a.nwg, 1e3f * ms / reps, reps);
    const char *lab[6] = {"line table", "A halo", "B mfma", "C voxels", "sums put", "row out"};
    for (int k = 0; k < 6 && !ph[k].empty(); ++k) {
        std::sort(ph[k].begin(), ph[k].end());
        printf("  %-12s %6lld  (p90 %lld)\n", lab[k], ph[k][ph[k].size() / 2], ph[k][ph[k].size() * 9 / 10]);
    }
    return 0;
}
