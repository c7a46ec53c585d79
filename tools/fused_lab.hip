// fused_lab.hip -- diagnostic build of the FUSED kernel with per-phase
// s_memtime stamps (thread 0 of every block), plus a timing of the plain
// engines.  Stamp values never reach an output; this binary is not the product.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/fused_lab tools/fused_lab.hip
//   run:   tools/fused_lab [n m batch]
#define BA_FUSED_STAMPS 1
#include "../byzantine-agreement_amd/csrc/ba_api.cpp"
#include "../byzantine-agreement_amd/csrc/ba_fused.hip"
#include "../byzantine-agreement_amd/csrc/ba_wave3.hip"
#include "../byzantine-agreement_amd/csrc/ba_wave4.hip"
#include "../byzantine-agreement_amd/csrc/ba_levels.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 10, m = argc > 2 ? atoi(argv[2]) : 3;
    const uint64_t B = argc > 3 ? strtoull(argv[3], nullptr, 0) : (1u << 20);
    ba_ctx* ctx = nullptr;
    if (ba_ctx_create(0, &ctx) != BA_OK) {
        fprintf(stderr, "ctx: %s\n", ba_last_error());
        return 1;
    }
    uint64_t *dec, *cnt;
    uint8_t* out;
    (void)hipMalloc(&dec, B * 8);
    (void)hipMalloc(&out, B);
    (void)hipMalloc(&cnt, 16 * 8);
    ba_params p{};
    p.n = n;
    p.m = m;
    p.seed = 0xBA5EED;
    p.faulty_mode = BA_FAULTY_RANDOM;
    p.f = (n - 1) / 3;
    p.order_mode = BA_ORDER_RANDOM;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (uint32_t eng : {(uint32_t)BA_ENGINE_FUSED, (uint32_t)BA_ENGINE_LEVELS}) {
        p.engine = eng;
        for (int i = 0; i < 3; ++i)
            if (ba_run_trials_device(ctx, &p, B, nullptr, nullptr, nullptr, nullptr, dec, out, cnt,
                                     nullptr) != BA_OK) {
                fprintf(stderr, "run: %s\n", ba_last_error());
                return 1;
            }
        (void)hipDeviceSynchronize();
        const int R = 10;
        (void)hipEventRecord(e0, ctx->stream);
        for (int i = 0; i < R; ++i)
            (void)ba_run_trials_device(ctx, &p, B, nullptr, nullptr, nullptr, nullptr, dec, out, cnt,
                                       nullptr);
        (void)hipEventRecord(e1, ctx->stream);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"engine\": %u, \"n\": %u, \"m\": %u, \"batch\": %llu, \"ms_per_call\": %.4f, "
               "\"trials_per_s\": %.4e}\n",
               eng, n, m, (unsigned long long)B, ms / R, B / (ms / R * 1e-3));
        if (eng == BA_ENGINE_FUSED) {
            std::vector<unsigned long long> st(kPartialRows * 8);
            (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_fused_stamps), st.size() * 8);
            GeoEntry* ge = ctx->geos.begin()->second.get();
            uint64_t blocks = 0;
            double ph[6] = {0}, tot = 0;
            for (uint64_t b = 0; b < (uint64_t)kPartialRows; ++b) {
                unsigned long long s = 0;
                for (int i = 0; i < 6; ++i) s += st[b * 8 + i];
                if (!s) continue;
                ++blocks;
                for (int i = 0; i < 6; ++i) ph[i] += (double)st[b * 8 + i];
            }
            for (int i = 0; i < 6; ++i) {
                ph[i] /= blocks ? blocks : 1;
                tot += ph[i];
            }
            printf("{\"fused_plan\": {\"wpb\": %u, \"threads\": %u, \"lds_bytes\": %u, "
                   "\"grid\": %llu}, \"phase_cycles_per_block\": {\"A_input\": %.0f, \"B_relay\": %.0f, "
                   "\"C_leaf\": %.0f, \"D_inner\": %.0f, \"E_root\": %.0f, \"E_trials\": %.0f, \"total\": %.0f}}\n",
                   ge->fp.wpb, ge->fp.threads, ge->fp.lds_bytes, (unsigned long long)blocks,
                   ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], tot);
        }
    }
    ba_ctx_destroy(ctx);
    return 0;
}
