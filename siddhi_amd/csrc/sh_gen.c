/* sh_gen.c — synthetic workloads of BASELINE.md (host, deterministic).
 *
 * RNG: splitmix64, seed 20261015 + config index. Timestamps: ms int64 from
 * t0 = 1_700_000_000_000 with ts_i = t0 + floor(i / R). Prices: per-key
 * geometric random walk, start U[15,45], x exp(N(0, 0.01)), rounded to 0.01,
 * stored as float. Volume U[1, 1e4]. Keys uniform over [0, n_keys).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

static inline uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double u01(uint64_t* s) { return (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }

/* returns 0 on success */
int sh_gen_stock(int64_t n, int32_t n_keys, int64_t rate_per_ms, uint64_t seed, int64_t t0, int64_t* ts,
                 int32_t* keys, float* price, int64_t* volume) {
    uint64_t s = seed;
    double* walk = (double*)malloc(sizeof(double) * (size_t)n_keys);
    if (!walk) return -1;
    for (int32_t k = 0; k < n_keys; k++) walk[k] = -1.0;
    for (int64_t i = 0; i < n; i++) {
        int32_t k = (int32_t)(splitmix64(&s) % (uint64_t)n_keys);
        double p = walk[k];
        if (p < 0) {
            p = 15.0 + 30.0 * u01(&s);
        } else {
            double u1 = u01(&s), u2 = u01(&s);
            if (u1 < 1e-300) u1 = 1e-300;
            double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2) * 0.01;
            p = p * exp(z);
        }
        p = floor(p * 100.0 + 0.5) / 100.0;
        if (p < 0.01) p = 0.01;
        walk[k] = p;
        ts[i] = t0 + i / rate_per_ms;
        keys[i] = k;
        price[i] = (float)p;
        if (volume) volume[i] = 1 + (int64_t)(splitmix64(&s) % 10000ull);
    }
    free(walk);
    return 0;
}

/* C5: card transactions. Cards uniform over [0, n_cards), amount lognormal(4, 1)
 * rounded to 0.01 (at least 0.01) and stored as float, merchant uniform over
 * [0, n_merchants), ts_i = t0 + floor(i / R). Returns 0 on success. */
int sh_gen_txn(int64_t n, int32_t n_cards, int32_t n_merchants, int64_t rate_per_ms, uint64_t seed, int64_t t0,
               int64_t* ts, int32_t* card, float* amount, int32_t* merchant) {
    uint64_t s = seed;
    for (int64_t i = 0; i < n; i++) {
        card[i] = (int32_t)(splitmix64(&s) % (uint64_t)n_cards);
        double u1 = u01(&s), u2 = u01(&s);
        if (u1 < 1e-300) u1 = 1e-300;
        const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        double a = floor(exp(4.0 + z) * 100.0 + 0.5) / 100.0;
        if (a < 0.01) a = 0.01;
        amount[i] = (float)a;
        merchant[i] = (int32_t)(splitmix64(&s) % (uint64_t)n_merchants);
        ts[i] = t0 + i / rate_per_ms;
    }
    return 0;
}
