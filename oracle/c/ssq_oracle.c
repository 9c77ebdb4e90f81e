/*
 * CPU oracle, plain C: scalar restatement of the reference's uniform affine
 * fake-quant and its 'max' / 'mse' scale initialisation.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ as a second checker and by bench.py's
 * cpu_baseline leg as the timed CPU port.  Never linked into libssq.so.
 *
 *   ssqo_fake_quant      quant_layer.py:92-98   (round_ste(x/delta)+zp, clamp, dequant)
 *   ssqo_init_max        quant_layer.py:124-142 (fp64 host math on fp32 extrema)
 *   ssqo_init_mse        quant_layer.py:144-175 (80 shrink candidates, mean |x-q|^2.4)
 *
 * Compile with -ffp-contract=off (no FMA): every fp32 operation rounds separately,
 * matching the reference's one-op-per-tensor evaluation.  Parity: tests/test_oracle_c.py
 * pins these against the golden vectors produced by the reference.
 */
#include <math.h>
#include <stdint.h>

void ssqo_fake_quant(const float* x, float* y, uint8_t* codes, const float* delta,
                     const float* zp, int64_t n, int64_t inner, int64_t nch, float scale,
                     int qmin, int qmax) {
  const float lo = (float)qmin, hi = (float)qmax;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t c = nch == 1 ? 0 : (i / inner) % nch;
    const float d = delta[c] * scale, z = zp[c];
    const float t = x[i] / d;
    float q = ((rintf(t) - t) + t) + z;  /* round_ste: round(t), NaN at t = +-inf */
    q = q < lo ? lo : (q > hi ? hi : q); /* torch.clamp: NaN stays NaN */
    y[i] = (q - z) * d;
    if (codes) codes[i] = q == q ? (uint8_t)((int)q & 0xff) : 0;
  }
}

void ssqo_init_max(const float* x, int64_t rows, int64_t inner, int n_bits, int sym,
                   float* delta, float* zp, float* raw_zp) {
  for (int64_t r = 0; r < rows; ++r) {
    const float* p = x + r * inner;
    float mn = p[0], mx = p[0];
    for (int64_t k = 1; k < inner; ++k) {
      mn = p[k] < mn ? p[k] : mn;
      mx = p[k] > mx ? p[k] : mx;
    }
    double x_min = mn < 0.0f ? (double)mn : 0.0, x_max = mx > 0.0f ? (double)mx : 0.0;
    if (sym) {
      const double a = fabs(x_min) > x_max ? fabs(x_min) : x_max;
      x_min = x_min < 0 ? -a : 0.0;
      x_max = a;
    }
    double d = (x_max - x_min) / (double)((1 << n_bits) - 1);
    if (d < 1e-8) d = 1e-8;
    delta[r] = (float)d;
    zp[r] = (float)rint(-x_min / d);
    raw_zp[r] = (float)(-x_min);
  }
}

void ssqo_init_mse(const float* x, int64_t rows, int64_t inner, int n_bits, int sym,
                   float* delta, float* zp, float* raw_zp) {
  const float hi = (float)((1 << n_bits) - 1);
  for (int64_t r = 0; r < rows; ++r) {
    const float* p = x + r * inner;
    float mn = p[0], mx = p[0];
    for (int64_t k = 1; k < inner; ++k) {
      mn = p[k] < mn ? p[k] : mn;
      mx = p[k] > mx ? p[k] : mx;
    }
    if (sym) {
      const float a = fabsf(mn) > mx ? fabsf(mn) : mx;
      mn = mn < 0.0f ? -a : 0.0f;
      mx = a;
    }
    double best = 1e10;
    delta[r] = zp[r] = raw_zp[r] = NAN;
    for (int i = 0; i < 80; ++i) {
      const float s = (float)(1.0 - (double)i * 0.01);
      const float nmax = mx * s, nmin = mn * s;
      const float d = (nmax - nmin) / hi;
      const float z = rintf(-nmin / d);
      double acc = 0.0;
      for (int64_t k = 0; k < inner; ++k) {
        float q = rintf(p[k] / d) + z;
        q = q < 0.0f ? 0.0f : (q > hi ? hi : q);
        const float e = fabsf(p[k] - (q - z) * d);
        acc += pow((double)e, 2.4);
      }
      const double score = acc / (double)inner;
      if (score < best) {
        best = score;
        delta[r] = d;
        zp[r] = sym ? 0.0f : z;
        raw_zp[r] = sym ? 0.0f : -nmin;
      }
    }
  }
}
