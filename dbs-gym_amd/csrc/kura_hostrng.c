// kura_hostrng.c -- libkura_host.so: the host draws of reset() for a whole
// batch of envs, in native code.
//
// The reference draws every reset's randomness from NumPy's legacy global
// RandomState (MT19937): SpatialKuramoto.__init__ seeds it with rand_seed
// (environment/env.py:291), reset() draws theta0 = normal(mean, sd, N)
// (env.py:595-597) and remove_negative_w0 draws randn(k) (utils.py:819-823);
// the driver's generate_w0_with_locus draws rand(N) and uniform(N)
// (utils.py:868, :927).  One numpy.random.RandomState per env costs ~0.17 ms
// to construct (its MT19937 is first seeded from OS entropy through a
// SeedSequence, then re-seeded) -- 0.7 s of host setup at 4096 envs -- and
// every draw is a separate Python call.  Here the B streams live in one array
// of kh_mt records (the fields of RandomState.get_state(): key, pos,
// has_gauss, cached_gaussian) and the draws of many envs are one call.
//
// Restated from the published algorithms NumPy implements (numpy 2.2 here):
//   * MT19937 (Matsumoto & Nishimura 1998): init_genrand seeding, the
//     624-word twist, the tempering;
//   * RandomState's legacy seeding of an integer seed: init_genrand(seed),
//     pos = 624, no cached Gaussian;
//   * random_sample: 53-bit doubles ((a >> 5) * 2^26 + (b >> 6)) / 2^53;
//   * uniform(low, high): low + (high - low) * random_sample;
//   * the legacy Gaussian (Marsaglia's polar method with one cached value):
//     randn = gauss, normal(loc, scale) = loc + scale * gauss.
// tests/test_hostrng.py checks every entry point bit for bit against
// numpy.random.RandomState on the same seeds, including the cached-Gaussian
// state carried across calls and get_state/set_state round trips.
//
// Plain C99, -ffp-contract=off (the products and sums must round as NumPy's
// own C does), libm's log/sqrt as NumPy calls them.
#include <math.h>
#include <stdint.h>
#include <string.h>

#define KH_N 624
#define KH_M 397

typedef struct {
    uint32_t key[KH_N];
    int32_t pos;
    int32_t has_gauss;
    double gauss;
} kh_mt;

static void kh_init_genrand(kh_mt* s, uint32_t seed) {
    s->key[0] = seed;
    for (int i = 1; i < KH_N; ++i) {
        const uint32_t p = s->key[i - 1];
        s->key[i] = 1812433253u * (p ^ (p >> 30)) + (uint32_t)i;
    }
    s->pos = KH_N;
    s->has_gauss = 0;
    s->gauss = 0.0;
}

static inline uint32_t kh_mix(uint32_t hi, uint32_t lo, uint32_t far) {
    const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1u)) & 0x9908b0dfu);
}

static void kh_twist(kh_mt* s) {
    uint32_t* k = s->key;
    int i = 0;
    for (; i < KH_N - KH_M; ++i) k[i] = kh_mix(k[i], k[i + 1], k[i + KH_M]);
    for (; i < KH_N - 1; ++i) k[i] = kh_mix(k[i], k[i + 1], k[i + KH_M - KH_N]);
    k[KH_N - 1] = kh_mix(k[KH_N - 1], k[0], k[KH_M - 1]);
    s->pos = 0;
}

static inline uint32_t kh_next32(kh_mt* s) {
    if (s->pos >= KH_N) kh_twist(s);
    uint32_t y = s->key[s->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

static inline double kh_double(kh_mt* s) {
    const uint32_t a = kh_next32(s) >> 5, b = kh_next32(s) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

static inline double kh_gauss1(kh_mt* s) {
    if (s->has_gauss) {
        const double t = s->gauss;
        s->has_gauss = 0;
        s->gauss = 0.0;
        return t;
    }
    double x1, x2, r2;
    do {
        x1 = 2.0 * kh_double(s) - 1.0;
        x2 = 2.0 * kh_double(s) - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = sqrt(-2.0 * log(r2) / r2);
    s->gauss = f * x1;
    s->has_gauss = 1;
    return f * x2;
}

int kh_state_size(void) { return (int)sizeof(kh_mt); }

// The batch entry points take distinct rows (one stream per row; the rows are
// drawn in parallel).
//
// streams[rows[i]] <- RandomState(seeds[i]) (0 <= seed < 2^32)
void kh_seed(kh_mt* streams, const int64_t* rows, const uint32_t* seeds, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) kh_init_genrand(&streams[rows[i]], seeds[i]);
}

// streams[row].randint(low, high) with size=None, 1 <= high - low <= 2^32:
// numpy's legacy bounded integers (random_bounded_uint64_fill, masked
// rejection on 32-bit draws; RandomState.choice(a) draws its index this way).
int64_t kh_randint(kh_mt* streams, int64_t row, int64_t low, int64_t high) {
    const uint64_t rng = (uint64_t)(high - 1 - low);
    if (rng == 0) return low;
    kh_mt* s = &streams[row];
    if (rng == 0xFFFFFFFFull) return low + (int64_t)kh_next32(s);
    uint64_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t val;
    while ((val = kh_next32(s) & (uint32_t)mask) > rng) {
    }
    return low + (int64_t)val;
}

// out[i, :m] <- streams[rows[i]].random_sample(m)
void kh_random_sample(kh_mt* streams, const int64_t* rows, int64_t n, int64_t m, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        kh_mt* s = &streams[rows[i]];
        double* o = out + i * m;
        for (int64_t j = 0; j < m; ++j) o[j] = kh_double(s);
    }
}

// out[i, :m] <- streams[rows[i]].uniform(low[i], high[i], m)
void kh_uniform(kh_mt* streams, const int64_t* rows, int64_t n, const double* low, const double* high, int64_t m,
                double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        kh_mt* s = &streams[rows[i]];
        const double lo = low[i], range = high[i] - low[i];
        double* o = out + i * m;
        for (int64_t j = 0; j < m; ++j) o[j] = lo + range * kh_double(s);
    }
}

// out[i, :m] <- streams[rows[i]].normal(loc[i], scale[i], m)
void kh_normal(kh_mt* streams, const int64_t* rows, int64_t n, const double* loc, const double* scale, int64_t m,
               double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        kh_mt* s = &streams[rows[i]];
        const double mu = loc[i], sd = scale[i];
        double* o = out + i * m;
        for (int64_t j = 0; j < m; ++j) o[j] = mu + sd * kh_gauss1(s);
    }
}

// out[:m] <- streams[row].randn(m)
void kh_randn(kh_mt* streams, int64_t row, int64_t m, double* out) {
    kh_mt* s = &streams[row];
    for (int64_t j = 0; j < m; ++j) out[j] = kh_gauss1(s);
}

// numpy's float64 add.reduce inner loop on a contiguous block (pairwise
// summation: blocks of <= 128 summed with 8 partial sums, halves split at a
// multiple of 8)
static double kh_pairwise_sum(const double* a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return kh_pairwise_sum(a, n2) + kh_pairwise_sum(a + n2, n - n2);
}

// remove_negative_w0 (utils.py:819-823) on row i of x (n rows of m, in
// place) with stream rows[i]: the k entries <= 0 (in index order) become
// |0.05 * randn(k)| + mean(x_i) (the mean of the row before the update);
// rows without such entries draw nothing.
void kh_remove_nonpositive(kh_mt* streams, const int64_t* rows, int64_t n, double* x, int64_t m) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double* r = x + i * m;
        int64_t k = 0;
        for (int64_t j = 0; j < m; ++j) k += (r[j] <= 0.0);
        if (k == 0) continue;
        kh_mt* s = &streams[rows[i]];
        // add.reduce runs its inner loop over buffers of 8192 elements
        double sum = 0.0;
        for (int64_t c = 0; c < m; c += 8192) sum += kh_pairwise_sum(r + c, m - c < 8192 ? m - c : 8192);
        const double mean = sum / (double)m;
        for (int64_t j = 0; j < m; ++j)
            if (r[j] <= 0.0) r[j] = fabs(kh_gauss1(s) * 0.05) + mean;
    }
}

// out[i] <- numpy.interp(x[i], xp, fp) for sorted xp (m >= 2): the largest j
// with xp[j] <= x, then fp[j] when x == xp[j] (or j is the last point),
// otherwise slope_j * (x - xp[j]) + fp[j] with slope_j = (fp[j+1] - fp[j]) /
// (xp[j+1] - xp[j]); x < xp[0] -> left, x > xp[m-1] -> right.  The inverse
// CDF of the w0 prior (model_setup.w0_from_uniform, utils.py:847-882) on B*N
// draws; OpenMP over the elements.
void kh_interp(const double* x, int64_t n, const double* xp, const double* fp, int64_t m, double left, double right,
               double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const double v = x[i];
        double r;
        if (v != v) {
            r = v;
        } else if (v < xp[0]) {
            r = left;
        } else if (v > xp[m - 1]) {
            r = right;
        } else {
            // the last index with xp <= v (xp[0] <= v here); branch-free
            // halving, the search is bound by mispredictions otherwise
            const double* base = xp;
            int64_t len = m;
            while (len > 1) {
                const int64_t half = len / 2;
                base = (base[half] <= v) ? base + half : base;
                len -= half;
            }
            const int64_t j = base - xp;
            if (j >= m - 1 || xp[j] == v) {
                r = fp[j];
            } else {
                const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
                r = slope * (v - xp[j]) + fp[j];
                if (r != r) {
                    r = slope * (v - xp[j + 1]) + fp[j + 1];
                    if (r != r && fp[j] == fp[j + 1]) r = fp[j];
                }
            }
        }
        out[i] = r;
    }
}

// numpy's float64 add.reduce of a contiguous vector (the inner loop over
// buffers of 8192 elements, each a pairwise sum), from 0.0
static double kh_reduce_sum(const double* a, int64_t n) {
    double sum = 0.0;
    for (int64_t c = 0; c < n; c += 8192) sum += kh_pairwise_sum(a + c, n - c < 8192 ? n - c : 8192);
    return sum;
}

// generate_perturbations (environment/env.py:21-57) of row i of initial
// (n rows of m) with stream rows[i]: out[i] (M+1 rows of m) = the random walk
// initial, initial + s*g_1, ... with s = step_scale * std(initial, ddof=1)
// (numpy's std: pairwise mean, squared deviations, pairwise sum / (m-1),
// sqrt) and g_k = randn(m).  tmp: n*m doubles of scratch.
void kh_perturbations(kh_mt* streams, const int64_t* rows, int64_t n, const double* initial, int64_t m, int64_t M,
                      double step_scale, double* out, double* tmp) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        kh_mt* s = &streams[rows[i]];
        const double* x = initial + i * m;
        double* o = out + i * (M + 1) * m;
        double* d = tmp + i * m;
        const double mean = kh_reduce_sum(x, m) / (double)m;
        for (int64_t j = 0; j < m; ++j) {
            const double v = x[j] - mean;
            d[j] = v * v;
        }
        const double var = kh_reduce_sum(d, m) / (double)(m - 1);
        const double sc = step_scale * sqrt(var);
        for (int64_t j = 0; j < m; ++j) o[j] = x[j];
        for (int64_t k = 1; k <= M; ++k) {
            const double* cur = o + (k - 1) * m;
            double* nxt = o + k * m;
            for (int64_t j = 0; j < m; ++j) nxt[j] = cur[j] + sc * kh_gauss1(s);
        }
    }
}
