/* C restatement of the build's synthetic fills (byzantine_aircomp_amd/csrc/oma.hip
 * fill_clients / fill_normal, philox.h normal4): Philox4x32-10 keyed (seed, stream,
 * iteration, index) and Box-Muller in double precision, rounded to float.
 *
 * TEST INFRASTRUCTURE ONLY (oracle/__init__.py): it rebuilds, on the CPU, the inputs the
 * GPU tests generate on the device, so tests/test_iteration_wellposed.py can check their
 * iteration counts for well-posedness at sizes the numpy restatement (oracle/philox.py,
 * which this file must agree with) is too slow for.  The device's fast sin/cos put its
 * values within ~1e-6 of these.
 *
 *   gcc -O2 -fopenmp -shared -fPIC oracle/philox_fill.c -o oracle/_philox_fill.so -lm
 */
#include <math.h>
#include <stdint.h>

#define STREAM_FILL 0x46494C4Cu

static void philox4x32_10(uint32_t c[4], uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

static double u01(uint32_t v) { return ((double)(v >> 8) + 1.0) / 16777216.0; }

/* normal z[j] of block (iter, idx) on stream: oracle/philox.py normal4 */
static void normal4(uint64_t seed, uint32_t stream, uint64_t iter, uint64_t idx, double z[4]) {
  uint32_t c[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)iter,
                   stream ^ (uint32_t)(iter >> 32)};
  philox4x32_10(c, seed);
  for (int h = 0; h < 2; ++h) {
    const double rad = sqrt(-2.0 * log(u01(c[2 * h]))), t = 2.0 * M_PI * u01(c[2 * h + 1]);
    z[2 * h] = rad * cos(t);
    z[2 * h + 1] = rad * sin(t);
  }
}

/* X[k][j] (row-major, ld = d): mu + sd * normal (c & 3) of block (k, c >> 2), c = col_off + j;
 * the last B rows take (mu_b, sd_b) */
void fill_clients(int64_t K, int64_t d, int64_t B, double mu_h, double sd_h, double mu_b,
                  double sd_b, uint64_t seed, int64_t col_off, float* X) {
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < K; ++k) {
    const int byz = k >= K - B;
    const double mu = byz ? mu_b : mu_h, sd = byz ? sd_b : sd_h;
    double z[4];
    int64_t cached = -1;
    for (int64_t j = 0; j < d; ++j) {
      const int64_t c = col_off + j;
      if ((c >> 2) != cached) {
        cached = c >> 2;
        normal4(seed, STREAM_FILL, (uint64_t)k, (uint64_t)cached, z);
      }
      X[k * d + j] = (float)(mu + sd * z[c & 3]);
    }
  }
}

/* v[i] = mu + sd * normal (c & 3) of block (0xFFFFFFFF, c >> 2), c = off + i */
void fill_normal(int64_t n, double mu, double sd, uint64_t seed, int64_t off, float* v) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t c = off + i;
    double z[4];
    normal4(seed, STREAM_FILL, 0xFFFFFFFFull, (uint64_t)(c >> 2), z);
    v[i] = (float)(mu + sd * z[c & 3]);
  }
}
