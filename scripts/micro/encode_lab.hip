// Lab harness: the real fused encode kernel (RS_STAMP build) on C3, reporting
// the in-kernel shader clock (s_memtime ticks / s_memrealtime at 100 MHz) and
// the mean wave lifetime.  Diagnostic only; never quote this build's time.
#define RS_STAMP 1
#include "../../reedsolomon16_amd/csrc/kernels.hip"
#include "../../reedsolomon16_amd/csrc/gf_host.cpp"
#include "../../reedsolomon16_amd/csrc/codec.cpp"
#include <cstdio>
#include <vector>

int main(int argc, char **argv) {
    const int k = 128, p = 32;
    const size_t S = 1 << 20;
    rs_codec *c = nullptr;
    if (rs_new(16, k, p, 0, &c)) return 1;
    uint8_t *slab;
    (void)hipMalloc(&slab, (size_t)(k + p) * S);
    (void)hipMemset(slab, 0x5A, (size_t)(k + p) * S);
    for (int i = 0; i < 5; i++) rs_encode_dev_batch(c, slab, S, (k + p) * S, 1, S, nullptr);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, c->stream);
    const int N = 20;
    for (int i = 0; i < N; i++) rs_encode_dev_batch(c, slab, S, (k + p) * S, 1, S, c->stream);
    (void)hipEventRecord(e1, c->stream);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> st(3 << 16);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_rs_stamps), st.size() * 8);
    const int NW = getenv("RS_NO_SPLIT") ? 2048 : 4096;  // waves of the C3 launch
    double cyc = 0, rt = 0;
    int n = 0;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int w = 0; w < NW; w++) {
        if (st[4 * w + 1] == 0) continue;
        cyc += st[4 * w];
        rt += st[4 * w + 1];
        n++;
        t0 = std::min(t0, st[4 * w + 2]);
        t1 = std::max(t1, st[4 * w + 2] + st[4 * w + 1]);
    }
    cyc /= n;
    rt /= n;
    // histogram of wave start times (us after the first start) and per-CU residency
    int hist[16] = {0};
    for (int w = 0; w < NW; w++) {
        double s0 = (st[4 * w + 2] - t0) / 100.0;
        int b = (int)(s0 / 5.0);
        hist[b < 15 ? b : 15]++;
    }
    printf("span first start -> last end: %.2f us\nwave start histogram (5 us bins):", (t1 - t0) / 100.0);
    for (int i = 0; i < 16; i++) printf(" %d", hist[i]);
    printf("\n");
    double f = 0, wt = 0, fft = 0, pre = 0;
    for (int w = 0; w < NW; w++) {
        f += st[32768 + 4 * w]; wt += st[32768 + 4 * w + 1]; fft += st[32768 + 4 * w + 2]; pre += st[32768 + 4 * w + 3];
    }
    printf("per wave (cycles): first-data wait %.0f | later chunk waits %.0f | IFFT phase total %.0f | FFT %.0f | after FFT %.0f\n",
           f / NW, wt / NW, pre / NW - f / NW - wt / NW, fft / NW, cyc - pre / NW - fft / NW);
    double ch[8] = {0}, cs[8] = {0};
    for (int w = 0; w < NW; w++)
        for (int c = 0; c < 4; c++) {
            ch[c] += st[65536 + 16 * w + 2 * c];
            cs[c] += st[65536 + 16 * w + 2 * c + 1];
        }
    printf("per chunk (cycles, incl. its top wait): ");
    for (int c = 0; c < 4; c++) printf(" c%d start %.0f dur %.0f |", c, cs[c] / NW, ch[c] / NW);
    printf("\n");
    {   // end-time histogram (5 us bins) and per-XCD mean wave life / last end
        int eh[20] = {0};
        double xl[8] = {0}, xe[8] = {0};
        int xn[8] = {0};
        for (int w = 0; w < NW; w++) {
            const double e = (st[4 * w + 2] + st[4 * w + 1] - t0) / 100.0;
            int b = (int)(e / 5.0);
            eh[b < 19 ? b : 19]++;
            const int x = (int)((st[4 * w + 3] >> 32) & 7);
            xl[x] += st[4 * w + 1] / 100.0;
            xn[x]++;
            if (e > xe[x]) xe[x] = e;
        }
        printf("wave end histogram (5 us bins):");
        for (int i = 0; i < 20; i++) printf(" %d", eh[i]);
        printf("\nper XCD: ");
        for (int x = 0; x < 8; x++) printf(" [%d] n=%d life %.1f last %.1f |", x, xn[x], xn[x] ? xl[x] / xn[x] : 0.0, xe[x]);
        printf("\n");
    }
    unsigned long long hw0 = st[3];
    printf("sample hw_id/xcc of wave0: xcc=%llu hwid=0x%llx\n", hw0 >> 32, hw0 & 0xffffffffull);
    printf("kernel %.2f us/launch; waves %d; mean wave life %.0f shader cycles = %.2f us; clock %.3f GHz\n",
           ms * 1e3 / N, n, cyc, rt / 100.0, cyc / (rt / 100.0) / 1e3);
    return 0;
}
