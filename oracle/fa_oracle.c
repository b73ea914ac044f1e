/*
 * fa_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker.  The product path (flearn_amd/) never links or calls it.
 *
 * A per-element, strictly sequential restatement of the reference's aggregation arithmetic,
 * compiled with -ffp-contract=off (SSE2 on x86-64: every float op is rounded to its own type):
 *
 *   Strategy.server_ensemble  flearn/common/strategy/strategy.py:102-130
 *       w = a0*x0                          (123)
 *       w += a_n*x_n   n = 1..N-1, in order (124-126)
 *       w = np.divide(w, np.sum(a))        (127-129)
 *     with the dtypes numpy (NEP 50) gives each step for the weight type — see
 *     include/flearn_amd.h FA_MODE_*;
 *   AVGM.mean_momentum        flearn/common/strategy/avgm.py:19-36
 *   OPT.adaptive_opt          flearn/common/strategy/opt.py:23-65 (adagrad / yogi / adam)
 *
 * Pinned against golden fixtures captured from the reference itself (tests/golden/).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- reduce: row-major sweep, per element identical to the sequential client loop ---- */

/* Python-float/int weights: fl32(a_n) * x in fp32, fp32 running sum, then f64 divide. */
void ora_reduce_w32_div64(const float* stack, int64_t stride, int32_t n, const float* w,
                          double denom, int64_t ncols, double* out64) {
  float* acc = (float*)malloc((size_t)(ncols > 0 ? ncols : 1) * sizeof(float));
  for (int64_t p = 0; p < ncols; ++p) acc[p] = w[0] * stack[p];
  for (int32_t i = 1; i < n; ++i) {
    const float* row = stack + (int64_t)i * stride;
    const float wi = w[i];
    for (int64_t p = 0; p < ncols; ++p) {
      const float prod = wi * row[p];
      acc[p] = acc[p] + prod;
    }
  }
  for (int64_t p = 0; p < ncols; ++p) out64[p] = (double)acc[p] / denom;
  free(acc);
}

/* np.float32 weights: everything fp32, divide by the fp32 np.sum. */
void ora_reduce_w32_div32(const float* stack, int64_t stride, int32_t n, const float* w,
                          float denom, int64_t ncols, float* out32) {
  float* acc = (float*)malloc((size_t)(ncols > 0 ? ncols : 1) * sizeof(float));
  for (int64_t p = 0; p < ncols; ++p) acc[p] = w[0] * stack[p];
  for (int32_t i = 1; i < n; ++i) {
    const float* row = stack + (int64_t)i * stride;
    for (int64_t p = 0; p < ncols; ++p) {
      const float prod = w[i] * row[p];
      acc[p] = acc[p] + prod;
    }
  }
  for (int64_t p = 0; p < ncols; ++p) out32[p] = acc[p] / denom;
  free(acc);
}

/* The ORDER of the opt-in split-N kernel (flearn_amd/csrc/fa_device.hpp reduce_kernel_splitn),
 * not the reference's: clients cut into `nsplit` contiguous splits [v*n/nsplit, (v+1)*n/nsplit),
 * each summed in list order from its first product (fl32(w*x) products, fp32 sums), combined by
 * the fixed tree ((p0+p1)+(p2+p3))+...  With `guard`, the kernel's cancellation guard: the sums
 * of |product| are formed the same way, and a column with !(A <= 2|S|) or !(|S| <= 3e38) takes
 * the sequential (reference-order) sum instead.  Returns the fp32 sums (the caller divides as
 * the mode does).  Used by the tests to pin that kernel bit for bit and to measure how far its
 * order lies from the reference's sequential sum. */
void ora_sum_w32_splitn(const float* stack, int64_t stride, int32_t n, const float* w, int32_t nsplit,
                        int64_t ncols, float* out, int32_t guard) {
  const size_t cells = (size_t)(ncols > 0 ? ncols : 1) * (size_t)nsplit;
  float* part = (float*)malloc(cells * sizeof(float));
  float* apart = (float*)malloc(cells * sizeof(float));
  for (int32_t v = 0; v < nsplit; ++v) {
    const int32_t r0 = (int32_t)((int64_t)v * n / nsplit), r1 = (int32_t)((int64_t)(v + 1) * n / nsplit);
    float* acc = part + (int64_t)v * ncols;
    float* aacc = apart + (int64_t)v * ncols;
    for (int64_t p = 0; p < ncols; ++p) {
      const float prod = r0 < r1 ? w[r0] * stack[(int64_t)r0 * stride + p] : 0.0f;
      acc[p] = prod;
      aacc[p] = fabsf(prod);
    }
    for (int32_t i = r0 + 1; i < r1; ++i) {
      const float* row = stack + (int64_t)i * stride;
      for (int64_t p = 0; p < ncols; ++p) {
        const float prod = w[i] * row[p];
        acc[p] = acc[p] + prod;
        aacc[p] = aacc[p] + fabsf(prod);
      }
    }
  }
  for (int32_t h = 1; h < nsplit; h *= 2)
    for (int32_t v = 0; v + h < nsplit; v += 2 * h)
      for (int64_t p = 0; p < ncols; ++p) {
        part[(int64_t)v * ncols + p] = part[(int64_t)v * ncols + p] + part[(int64_t)(v + h) * ncols + p];
        apart[(int64_t)v * ncols + p] = apart[(int64_t)v * ncols + p] + apart[(int64_t)(v + h) * ncols + p];
      }
  for (int64_t p = 0; p < ncols; ++p) {
    const float sum = part[p], ab = fabsf(sum), two_ab = 2.0f * ab;
    const int flag = guard && (!(apart[p] <= two_ab) || !(ab <= 3.0e38f));
    if (flag) {  /* the reference's sequential sum */
      float acc = w[0] * stack[p];
      for (int32_t i = 1; i < n; ++i) {
        const float prod = w[i] * stack[(int64_t)i * stride + p];
        acc = acc + prod;
      }
      out[p] = acc;
    } else {
      out[p] = sum;
    }
  }
  free(part);
  free(apart);
}

/* np.float64 / np.int64 weights on fp32 tensors: promoted to f64 for product and sum. */
void ora_reduce_w64(const float* stack, int64_t stride, int32_t n, const double* w, double denom,
                    int64_t ncols, double* out64) {
  double* acc = (double*)malloc((size_t)(ncols > 0 ? ncols : 1) * sizeof(double));
  for (int64_t p = 0; p < ncols; ++p) acc[p] = w[0] * (double)stack[p];
  for (int32_t i = 1; i < n; ++i) {
    const float* row = stack + (int64_t)i * stride;
    for (int64_t p = 0; p < ncols; ++p) {
      const double prod = w[i] * (double)row[p];
      acc[p] = acc[p] + prod;
    }
  }
  for (int64_t p = 0; p < ncols; ++p) out64[p] = acc[p] / denom;
  free(acc);
}

/* f64 tensors (or int64 buffers promoted to f64). */
void ora_reduce_f64(const double* stack, int64_t stride, int32_t n, const double* w, double denom,
                    int64_t ncols, double* out64) {
  for (int64_t p = 0; p < ncols; ++p) out64[p] = w[0] * stack[p];
  for (int32_t i = 1; i < n; ++i) {
    const double* row = stack + (int64_t)i * stride;
    for (int64_t p = 0; p < ncols; ++p) {
      const double prod = w[i] * row[p];
      out64[p] = out64[p] + prod;
    }
  }
  for (int64_t p = 0; p < ncols; ++p) out64[p] = out64[p] / denom;
}

/* int64 buffers with Python-int weights: wrapping int64 arithmetic, then true divide. */
void ora_reduce_i64(const int64_t* stack, int64_t stride, int32_t n, const int64_t* w,
                    double denom, int64_t ncols, double* out64) {
  uint64_t* acc = (uint64_t*)malloc((size_t)(ncols > 0 ? ncols : 1) * sizeof(uint64_t));
  for (int64_t p = 0; p < ncols; ++p) acc[p] = (uint64_t)w[0] * (uint64_t)stack[p];
  for (int32_t i = 1; i < n; ++i) {
    const int64_t* row = stack + (int64_t)i * stride;
    for (int64_t p = 0; p < ncols; ++p) acc[p] += (uint64_t)w[i] * (uint64_t)row[p];
  }
  for (int64_t p = 0; p < ncols; ++p) out64[p] = (double)(int64_t)acc[p] / denom;
  free(acc);
}

/* ---- optimizer updates (ops as in include/flearn_amd.h FA_OP_*) ---- */
enum { ORA_AVGM = 1, ORA_ADAGRAD = 2, ORA_YOGI = 3, ORA_ADAM = 4 };

#define ORA_SIGN(x) ((x) > 0 ? 1 : ((x) < 0 ? -1 : ((x) == 0 ? 0 : (x))))

/* w_glob g (f64), w_local l (fp32 -> f64), state v (f64), in place; out = new w_local (f64). */
void ora_update_f64(int32_t op, const double* g, const float* l32, double* v, double beta,
                    double eta, double tau, double beta2, int64_t n, double* out) {
  const double c = 1.0 - beta2;
  for (int64_t p = 0; p < n; ++p) {
    const double l = (double)l32[p];
    const double d = g[p] - l;
    if (op == ORA_AVGM) {
      const double bv = beta * v[p];
      v[p] = d + bv;
      out[p] = l + v[p];
      continue;
    }
    const double m = d * d;
    if (op == ORA_ADAGRAD) {
      v[p] = v[p] + m;
    } else if (op == ORA_YOGI) {
      const double cm = c * m;
      const double s = ORA_SIGN(v[p] - m);
      const double t = cm * s;
      v[p] = v[p] - t;
    } else {
      const double a = beta2 * v[p];
      const double b = c * m;
      v[p] = a + b;
    }
    const double num = eta * d;
    const double den = sqrt(v[p]) + tau;
    const double step = num / den;
    out[p] = l + step;
  }
}

/* Same in fp32 (np.float32 weights make w_glob, delta and v_t float32 arrays). */
void ora_update_f32(int32_t op, const float* g, const float* l, float* v, double beta_d,
                    double eta_d, double tau_d, double beta2_d, int64_t n, float* out) {
  const float beta = (float)beta_d, eta = (float)eta_d, tau = (float)tau_d, beta2 = (float)beta2_d;
  const float c = (float)(1.0 - beta2_d);
  for (int64_t p = 0; p < n; ++p) {
    const float d = g[p] - l[p];
    if (op == ORA_AVGM) {
      const float bv = beta * v[p];
      v[p] = d + bv;
      out[p] = l[p] + v[p];
      continue;
    }
    const float m = d * d;
    if (op == ORA_ADAGRAD) {
      v[p] = v[p] + m;
    } else if (op == ORA_YOGI) {
      const float cm = c * m;
      const float s = ORA_SIGN(v[p] - m);
      const float t = cm * s;
      v[p] = v[p] - t;
    } else {
      const float a = beta2 * v[p];
      const float b = c * m;
      v[p] = a + b;
    }
    const float num = eta * d;
    const float den = sqrtf(v[p]) + tau;
    const float step = num / den;
    out[p] = l[p] + step;
  }
}

/* FedDyn (dyn.py:17-36), f64 w_glob: d = g*N - theta; h = fl32(h - (alpha/N)*d) computed in f64;
 * w = g - fl32(fl32(alpha)*h); theta = w.  h and theta are updated in place. */
void ora_update_dyn_f64(const double* g, float* h, double* theta, double nclients, double alpha,
                        int64_t n, double* out) {
  const double c = alpha / nclients;
  const float a32 = (float)alpha;
  for (int64_t p = 0; p < n; ++p) {
    const double gn = g[p] * nclients;
    const double d = gn - theta[p];
    const double cd = c * d;
    const float hn = (float)((double)h[p] - cd);
    const float ah = a32 * hn;
    const double w = g[p] - (double)ah;
    h[p] = hn;
    theta[p] = w;
    out[p] = w;
  }
}

/* Same with float32 w_glob (np.float32 weights): everything in fp32, c = fl32(alpha/N). */
void ora_update_dyn_f32(const float* g, float* h, float* theta, double nclients_d, double alpha_d,
                        int64_t n, float* out) {
  const float nclients = (float)nclients_d, c = (float)(alpha_d / nclients_d), a32 = (float)alpha_d;
  for (int64_t p = 0; p < n; ++p) {
    const float gn = g[p] * nclients;
    const float d = gn - theta[p];
    const float cd = c * d;
    const float hn = h[p] - cd;
    const float ah = a32 * hn;
    const float w = g[p] - ah;
    h[p] = hn;
    theta[p] = w;
    out[p] = w;
  }
}

/* ---- synthetic generator, identical to the device fill (flearn_amd/csrc/fa_reduce.hip) ---- */
static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void ora_fill_uniform(float* dst, int64_t stride, int32_t n_rows, int64_t ncols, uint64_t seed,
                      int64_t row0, int64_t colg0) {
  for (int32_t r = 0; r < n_rows; ++r) {
    const uint64_t key_row = (seed * 0xD1B54A32D192ED03ull) ^ ((uint64_t)(row0 + r) << 40);
    float* out = dst + (int64_t)r * stride;
    for (int64_t c = 0; c < ncols; ++c) {
      const uint64_t h = splitmix64(key_row ^ (uint64_t)(colg0 + c));
      out[c] = (float)(h >> 40) * 0x1.0p-23f - 1.0f;
    }
  }
}
