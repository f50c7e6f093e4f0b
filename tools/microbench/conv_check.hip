// v5 vs v6 (or the variant named by argv[2] as conv flags, e.g. 12 = v7) on the same random g8 activations / blocked weights (one conv, residual on):
// reports max |diff| of the 16-bit outputs and where the mismatches are.
#include "../../alphazero-multi-game_amd/csrc/conv_bf16.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 64, FL = argc > 2 ? atoi(argv[2]) : 4, C = 256, N = 256, HW = 225;
    const size_t act = (size_t)B * HW * C;
    std::vector<uint16_t> hA(act + AZ_ACT_TAIL, 0), hR(act + AZ_ACT_TAIL, 0), hW((size_t)9 * C * N);
    std::vector<int8_t> hQ(act, 0);
    std::vector<float> hb(N);
    srand(1);
    auto h16 = [](float f) { _Float16 x = (_Float16)f; uint16_t h; __builtin_memcpy(&h, &x, 2); return h; };
    for (size_t i = 0; i < act; ++i) { hA[i] = h16((rand() % 2001 - 1000) / 1000.0f); hR[i] = h16((rand() % 2001 - 1000) / 1000.0f); }
    for (auto& w : hW) w = h16((rand() % 2001 - 1000) / 16000.0f);
    for (auto& x : hb) x = (rand() % 2001 - 1000) / 1000.0f;
    uint16_t *dA, *dR, *dW, *dO5, *dO6, *dZ; int8_t *dQ, *dQ5, *dQ6; float* db;
    hipMalloc(&dA, hA.size() * 2); hipMalloc(&dR, hR.size() * 2); hipMalloc(&dW, hW.size() * 2);
    hipMalloc(&dO5, act * 2); hipMalloc(&dO6, act * 2); hipMalloc(&dZ, 256); hipMalloc(&dQ, act); hipMalloc(&dQ5, act); hipMalloc(&dQ6, act);
    hipMalloc(&db, N * 4);
    hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice); hipMemcpy(dR, hR.data(), hR.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW, hW.data(), hW.size() * 2, hipMemcpyHostToDevice); hipMemcpy(db, hb.data(), N * 4, hipMemcpyHostToDevice);
    hipMemset(dZ, 0, 256); hipMemset(dQ, 0, act); hipMemset(dO5, 0, act * 2); hipMemset(dO6, 0, act * 2);
    ConvBf16Args a{};
    a.Ahi = dA; a.Bblk = dW; a.Chi = dO5; a.Cq = dQ5; a.bias = db; a.Rhi = dR; a.Rq = dQ;
    a.M = B * HW; a.N = N; a.C = C; a.H = 15; a.W = 15; a.rows_per_sample = HW; a.relu = 1; a.zero = dZ; a.stamp = -1;
    az_diag_set_conv_flags(0);
    az_conv_g8_launch(a, 2, 0);
    a.Chi = dO6; a.Cq = dQ6;
    az_diag_set_conv_flags(FL);
    az_conv_g8_launch(a, 2, 0);
    hipDeviceSynchronize();
    std::vector<uint16_t> o5(act), o6(act);
    hipMemcpy(o5.data(), dO5, act * 2, hipMemcpyDeviceToHost); hipMemcpy(o6.data(), dO6, act * 2, hipMemcpyDeviceToHost);
    auto f = [](uint16_t h) { _Float16 x; __builtin_memcpy(&x, &h, 2); return (float)x; };
    // CPU reference (fp32 over the fp16 operands) for boards 0..1: which outputs does each kernel get right?
    {
        const int GI = C / 8;
        double e5 = 0, e6 = 0; int bad6 = 0; int badrow[15] = {0}, badcol[16] = {0}, badgrp[4] = {0};
        for (int b = 0; b < 2; ++b)
            for (int pix = 0; pix < 225; ++pix)
                for (int n = 0; n < N; ++n) {
                    const int y = pix / 15, x = pix % 15;
                    double acc = hb[n];
                    for (int tap = 0; tap < 9; ++tap) {
                        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
                        if (yy < 0 || yy > 14 || xx < 0 || xx > 14) continue;
                        const int q = yy * 15 + xx;
                        for (int ci = 0; ci < C; ++ci)
                            acc += (double)f(hW[((((size_t)(ci / 16) * 9 + tap) * 2 + (ci / 8) % 2) * N + n) * 8 + ci % 8]) *
                                   f(hA[(((size_t)b * GI + ci / 8) * 225 + q) * 8 + ci % 8]);
                    }
                    acc += f(hR[(((size_t)b * (N / 8) + n / 8) * 225 + pix) * 8 + n % 8]);
                    if (acc < 0) acc = 0;
                    const size_t e = (((size_t)b * (N / 8) + n / 8) * 225 + pix) * 8 + n % 8;
                    const double d5 = fabs(f(o5[e]) - acc), d6 = fabs(f(o6[e]) - acc);
                    e5 = fmax(e5, d5 / fmax(1.0, fabs(acc)));
                    e6 = fmax(e6, d6 / fmax(1.0, fabs(acc)));
                    if (d6 > 2e-2 * fmax(1.0, fabs(acc))) { ++bad6; badrow[y]++; badcol[x]++; badgrp[(n % 64) / 16]++; }
                }
        printf("vs CPU (2 boards): v5 max rel err %.3g, v6 max rel err %.3g, v6 bad %d of %d\n", e5, e6, bad6, 2 * 225 * N);
        printf("v6 bad by output row y:"); for (int i = 0; i < 15; ++i) printf(" %d", badrow[i]); printf("\n");
        printf("v6 bad by output col x:"); for (int i = 0; i < 15; ++i) printf(" %d", badcol[i]); printf("\n");
        printf("v6 bad by 16-col tile within 64:"); for (int i = 0; i < 4; ++i) printf(" %d", badgrp[i]); printf("\n");
    }
    double mx = 0; size_t nbad = 0; int hist_g[32] = {0}, hist_p[225] = {0};
    for (size_t i = 0; i < act; ++i) {
        const double d = fabs(f(o5[i]) - f(o6[i]));
        if (d > mx) mx = d;
        if (d > 1e-2) { ++nbad; const size_t e = i / 8; hist_p[e % 225]++; hist_g[(e / 225) % 32]++; }
    }
    printf("B=%d: max|v5-v6| = %g, %zu of %zu elements off by > 1e-2\n", B, mx, nbad, act);
    printf("bad by channel group:"); for (int g = 0; g < 32; ++g) printf(" %d", hist_g[g]); printf("\n");
    printf("bad by pixel (first 45):"); for (int p = 0; p < 45; ++p) printf(" %d", hist_p[p]); printf("\n");
    return 0;
}
