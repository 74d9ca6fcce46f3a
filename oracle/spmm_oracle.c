/*
 * CPU ORACLE -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Plain-C restatement of the reference's GCN aggregation
 *     output = torch.spmm(adj, support) + bias        (GCN/GCN.py:43-45)
 * over the CSR form of the reference adjacency (GCN/data_utils.py:63-70), with
 * double-precision accumulation per output row.  Used by bench.py as the
 * `cpu_baseline` ("port") leg, timed on the GPU box's host cores, and by the
 * tests as a fast checker at sizes the numpy oracle is too slow for.
 * Parity of this restatement is pinned against the reference-generated golden
 * vectors in tests/golden/ (tests/test_oracle_golden.py).
 */
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* Y[r,:] = sum_e val[e] * X[col[e],:] (+ bias) for rows [row0, row1). */
void oracle_spmm_csr(const int64_t* rowptr, const int32_t* col, const float* val, int64_t row0,
                     int64_t row1, const float* x, int64_t ldx, int64_t feat, const float* bias,
                     float* y, int64_t ldy) {
#pragma omp parallel
  {
    double* acc = (double*)malloc(sizeof(double) * (size_t)(feat > 0 ? feat : 1));
#pragma omp for schedule(dynamic, 256)
    for (int64_t r = row0; r < row1; ++r) {
      for (int64_t f = 0; f < feat; ++f) acc[f] = 0.0;
      for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
        const double w = (double)val[e];
        const float* xr = x + (int64_t)col[e] * ldx;
        for (int64_t f = 0; f < feat; ++f) acc[f] += w * (double)xr[f];
      }
      float* yr = y + (r - row0) * ldy;
      for (int64_t f = 0; f < feat; ++f) yr[f] = (float)(acc[f] + (bias ? (double)bias[f] : 0.0));
    }
    free(acc);
  }
}
