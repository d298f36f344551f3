/* Sanitizer driver for the CPU oracle (test infrastructure, like bgoracle.c).
 * Built by `make -C oracle asan` with -fsanitize=address,undefined and run by
 * tests/test_oracle_properties.py::test_oracle_under_asan: seeded random games
 * (valid and invalid actions, game-over resets, match ends) and move generation
 * on random / spread positions with every roll, checking checker conservation.
 * Any out-of-bounds access, leak or UB aborts with a report. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bgoracle.c"

static uint32_t lcg(uint32_t* s) { *s = *s * 1664525u + 1013904223u; return *s >> 8; }

static int count_side(const int8_t* x, int p) {
    int n = x[48 + p] + x[50 + p];
    for (int i = 0; i < 24; ++i) n += x[24 * p + i];
    return n;
}

int main(int argc, char** argv) {
    const int games = argc > 1 ? atoi(argv[1]) : 60;
    float obs[198];
    int8_t b52[52];
    int32_t st[9];
    long steps = 0;
    for (int g = 0; g < games; ++g) {
        void* e = calloc(1, (size_t)bgo_env_size());
        bgo_env_init(e, g % 3 ? 15 : 3, 500, (uint32_t)g);
        bgo_env_reset(e, obs);
        uint32_t rs = 77u + (uint32_t)g;
        for (int t = 0; t < 2000; ++t) {
            bgo_env_state(e, b52, st);
            if (count_side(b52, 0) != 15 || count_side(b52, 1) != 15) { fprintf(stderr, "checkers not conserved\n"); return 2; }
            const int n = st[3];
            int a = n ? (int)(lcg(&rs) % (uint32_t)n) : (int)(lcg(&rs) % 500u);
            if (n && lcg(&rs) % 50u == 0) a = n + (int)(lcg(&rs) % 3u);     /* invalid action */
            float r; int done, info[4];
            bgo_env_step(e, a, obs, &r, &done, info);
            ++steps;
            if (done) bgo_env_reset(e, obs);
        }
        bgo_env_free(e);
        free(e);
    }
    /* move generation on spread boards (> 500 moves) with every roll, small cap (truncation) */
    uint64_t* out = (uint64_t*)malloc(sizeof(uint64_t) * 64);
    for (int p = 0; p < 2; ++p)
        for (int r0 = 1; r0 <= 6; ++r0)
            for (int r1 = 1; r1 <= 6; ++r1) {
                memset(b52, 0, sizeof b52);
                for (int i = 0; i < 15; ++i) b52[24 * p + (p ? 23 - i : i)] = 1;
                b52[24 * (1 - p) + (p ? 0 : 23)] = 15;
                int nu = 0;
                const int n = bgo_movegen(b52, p, r0, r1, out, 64, &nu);
                if (n < 0) return 3;
            }
    free(out);
    printf("asan ok: %ld env steps, %d games\n", steps, games);
    return 0;
}
