// CPU check of the exactness argument behind fb_chain_scan and fb_long_chain (simgrid_amd/csrc/lmm_fb_kernels.hpp):
// the wave algorithm (64 lanes x 8 increments) and the workgroup algorithm (256 threads x 8 = 2048 increments,
// a block-wide int64 scan), emulated here lane by lane with the same integer arithmetic (the int64 prefix wraps
// like the device's when a step holds many out-of-binade sentinels 2^52), must
// give, bit for bit, the value of the sequential loop `rem -= d[k]` followed by the end clamp, on random
// batches built to hit ties (d / u = xx.5), binade crossings, exact landings on 2^e, tiny and huge
// increments and values that drop below the precision.  Prints the number of batches checked; exit 1 on a
// mismatch.  (Built and run by tests/test_fb_chain_scan.py.)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

static double seq(const double* d, int n, double x, double prec) {
  for (int k = 0; k < n; k++)
    x -= d[k];
  return x < prec ? 0.0 : x;
}

// the device algorithm, W lanes emulated (64: fb_chain_scan, 256: fb_long_chain); returns the value and sets
// *kout like the kernels
static long long wrap_add(long long a, long long b) {  // the device's int64 adds (two's complement wrap)
  return (long long)((unsigned long long)a + (unsigned long long)b);
}

static double scan(const double* d, int n, double x, double prec, int* kout, int W) {
  const int P = 8;
  int k = 0, exits = 0;
  while (k < n) {
    if (!(x >= prec)) { k = n; x = 0.0; break; }
    if (x < 0x1p-1022 || exits >= 12) break;
    int ex2;
    std::frexp(x, &ex2);
    const int e = ex2 - 1;
    const long long M = (long long)(std::ldexp(x, 52 - e) - 0x1p52);
    static long long incl[256][8], tot[256];
    static bool tie[256][8];
    for (int l = 0; l < W; l++) {
      long long run = 0;
      for (int t = 0; t < P; t++) {
        const int j = l * P + t;
        long long q = 0;
        tie[l][t] = false;
        if (j >= k && j < n) {
          const double sc = std::ldexp(d[j], 52 - e);
          if (!(sc < 0x1p52)) q = 1ll << 52;
          else {
            const double f = std::floor(sc), fr = sc - f;
            tie[l][t] = fr == 0.5;
            q = (long long)f + (fr > 0.5 ? 1 : 0);
          }
        }
        run = wrap_add(run, q);
        incl[l][t] = run;
      }
      tot[l] = run;
    }
    static long long exl[256];
    long long acc = 0;
    for (int l = 0; l < W; l++) { exl[l] = acc; acc = wrap_add(acc, tot[l]); }
    int js = -1;
    long long pb = 0;
    for (int l = 0; l < W && js < 0; l++)
      for (int t = 0; t < P; t++) {
        const int j = l * P + t;
        if (j >= k && j < n && (tie[l][t] || wrap_add(exl[l], incl[l][t]) >= M)) {
          js = j;
          pb = wrap_add(exl[l], t ? incl[l][t - 1] : 0);
          break;
        }
      }
    const double u = std::ldexp(1.0, e - 52);
    if (js < 0) { x -= double(acc) * u; k = n; break; }
    x -= double(pb) * u;
    x -= d[js];
    k = js + 1;
    exits++;
  }
  if (k >= n && x < prec)  // the batch's end clamp
    x = 0.0;
  *kout = k;
  return x;
}

int main(int argc, char** argv) {
  const long batches = argc > 1 ? std::atol(argv[1]) : 200000;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  static double d[2048];
  long fast = 0, sat = 0;
  for (long b = 0; b < batches; b++) {
    const int W = (b & 1) ? 256 : 64;  // fb_long_chain's 256 x 8 steps / fb_chain_scan's 64 x 8 batches
    const int n = 1 + int(g() % (8 * W));
    const int mode = int(g() % 7);
    double x = std::ldexp(1.0 + U(g), int(g() % 80) - 20);
    const double prec = (g() % 3 == 0) ? 1e-5 : std::ldexp(1.0, -60);
    if (mode == 5) x = std::ldexp(1.0, int(g() % 40));  // exactly a power of two
    int ex2;
    std::frexp(x, &ex2);
    const double u = std::ldexp(1.0, ex2 - 1 - 52);
    for (int i = 0; i < n; i++) {
      switch (mode) {
        case 0: d[i] = x * U(g) / n; break;                                       // drains the value
        case 1: d[i] = x * U(g) * 1e-6; break;                                    // stays in the binade
        case 2: d[i] = u * (double(g() % 64) + ((g() & 1) ? 0.5 : 0.25)); break;  // ties and quarter-ulps
        case 3: d[i] = (g() % 4 == 0) ? x * U(g) : u * double(g() % 8) * 0.5; break;
        case 4: d[i] = std::ldexp(U(g), int(g() % 120) - 100) * x; break;        // tiny to large
        case 6: d[i] = std::ldexp(1.0, ex2 - 1) * (1.0 + U(g)); break;           // every one >= 2^e: sentinels
        default: d[i] = u * double(g() % 3); break;                               // lands on 2^e
      }
    }
    if (mode == 6 && n >= 2048)
      sat++;  // a full step of 2048 sentinels: the int64 prefix wraps past 2^63
    int k = 0;
    double y = scan(d, n, x, prec, &k, W);
    if (k < n) {  // fallback: lane 0's loop with a clamp per step from k (the device does the same)
      for (int i = k; i < n; i++) { y -= d[i]; if (y < prec) y = 0.0; }
      if (k == 0) y = seq(d, n, x, prec);
    } else {
      fast++;
    }
    const double ref = seq(d, n, x, prec);
    if (std::memcmp(&y, &ref, sizeof y) != 0) {
      std::printf("MISMATCH batch %ld W %d mode %d n %d x %.17g: scan %.17g seq %.17g (k %d)\n", b, W, mode, n, x, y,
                  ref, k);
      return 1;
    }
  }
  // the saturated case once more, deterministic: 2048 increments of 2^e each, W = 256
  {
    const double x = 1.5, prec = 1e-5;
    for (int i = 0; i < 2048; i++) d[i] = 1.0;
    int k = 0;
    double y = scan(d, 2048, x, prec, &k, 256);
    for (int i = k; i < 2048; i++) { y -= d[i]; if (y < prec) y = 0.0; }
    const double ref = seq(d, 2048, x, prec);
    if (std::memcmp(&y, &ref, sizeof y) != 0) {
      std::printf("MISMATCH saturated step: scan %.17g seq %.17g (k %d)\n", y, ref, k);
      return 1;
    }
  }
  std::printf("ok %ld batches, %ld fully wave-parallel, %ld full sentinel steps\n", batches, fast, sat);
  return 0;
}
