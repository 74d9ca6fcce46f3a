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
#include <math.h>
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

/*
 * Both GAT layers over CSR for H heads at once (float64), rows [row0, row1):
 *   dense  (GAT/models/layers.py:25-32):  out_i = sum_j softmax_j(LeakyReLU(el_i + er_j)) Wh_j
 *   sparse (GAT/models/layers.py:105-122): out_i = sum_j e_ij Wh_j / sum_j e_ij,
 *                                           e_ij = exp(-LeakyReLU(el_i + er_j)), no max shift
 * No activation. A row without edges is written as NaN (dense: the caller fills the
 * reference's uniform average; sparse: the reference's 0/0). el/er rows have stride lde.
 * Same arithmetic as oracle/gnn_oracle.py:gat_csr, in C for full-size checks and the
 * multi-core cpu_baseline of bench.py's GAT line.
 */
void oracle_gat_csr(const int64_t* rowptr, const int32_t* col, int64_t row0, int64_t row1,
                    const float* wh, int64_t ldwh, const float* el, const float* er, int64_t lde,
                    int64_t heads, int64_t fh, double slope, int sparse, float* y, int64_t ldy) {
  const int64_t feat = heads * fh;
#pragma omp parallel
  {
    double* acc = (double*)malloc(sizeof(double) * (size_t)(feat > 0 ? feat : 1));
    double* den = (double*)malloc(sizeof(double) * (size_t)(heads > 0 ? heads : 1));
    double* mx = (double*)malloc(sizeof(double) * (size_t)(heads > 0 ? heads : 1));
#pragma omp for schedule(dynamic, 256)
    for (int64_t r = row0; r < row1; ++r) {
      float* yr = y + (r - row0) * ldy;
      const int64_t e0 = rowptr[r], e1 = rowptr[r + 1];
      if (e0 == e1) {
        for (int64_t f = 0; f < feat; ++f) yr[f] = (float)NAN;
        continue;
      }
      for (int64_t f = 0; f < feat; ++f) acc[f] = 0.0;
      for (int64_t h = 0; h < heads; ++h) {
        den[h] = 0.0;
        mx[h] = -INFINITY;
        if (!sparse) {
          for (int64_t e = e0; e < e1; ++e) {
            double s = (double)el[r * lde + h] + (double)er[(int64_t)col[e] * lde + h];
            s = s > 0 ? s : slope * s;
            if (s > mx[h]) mx[h] = s;
          }
        }
      }
      for (int64_t e = e0; e < e1; ++e) {
        const int64_t c = col[e];
        for (int64_t h = 0; h < heads; ++h) {
          double s = (double)el[r * lde + h] + (double)er[c * lde + h];
          s = s > 0 ? s : slope * s;
          const double p = sparse ? exp(-s) : exp(s - mx[h]);
          den[h] += p;
          const float* w = wh + c * ldwh + h * fh;
          for (int64_t f = 0; f < fh; ++f) acc[h * fh + f] += p * (double)w[f];
        }
      }
      for (int64_t h = 0; h < heads; ++h)
        for (int64_t f = 0; f < fh; ++f) yr[h * fh + f] = (float)(acc[h * fh + f] / den[h]);
    }
    free(acc);
    free(den);
    free(mx);
  }
}

/*
 * Fused gather + argmax over the neighbours (graph_utils.py:7-8, Aggregator 'MAX':
 * torch.argmax(neigh_feat, dim=1)): out[m, f] = the first j < k whose table[idx[m, j], f] is
 * the maximum under torch's order (a NaN is larger than every number; the first NaN wins).
 */
void oracle_sage_argmax(const float* table, int64_t ldt, const int64_t* idx, int64_t ldi,
                        int64_t M, int64_t k, int64_t feat, int64_t* out, int64_t ldo) {
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t m = 0; m < M; ++m) {
    for (int64_t f = 0; f < feat; ++f) {
      int64_t best = 0;
      float bv = table[idx[m * ldi] * ldt + f];
      for (int64_t j = 1; j < k && bv == bv; ++j) {
        const float v = table[idx[m * ldi + j] * ldt + f];
        if (v != v || v > bv) {
          best = j;
          bv = v;
        }
      }
      out[m * ldo + f] = best;
    }
  }
}

/*
 * Fused gather + neighbour reduction (GraphSAGE/GraphSAGE.py:47-49 + graph_utils.py:6):
 * out[m] = reduce_j table[idx[m*ldi + j]] over j < k, float64 accumulation.
 * mode 0 mean (torch.mean), 2 sum (NeighborAggregator 'sum'), 3 max-pool
 * (torch.max(dim=1).values: a NaN anywhere in the slice gives NaN).
 */
void oracle_sage_gather(const float* table, int64_t ldt, const int64_t* idx, int64_t ldi,
                        int64_t M, int64_t k, int64_t feat, int mode, float* out, int64_t ldo) {
#pragma omp parallel
  {
    double* acc = (double*)malloc(sizeof(double) * (size_t)(feat > 0 ? feat : 1));
#pragma omp for schedule(dynamic, 256)
    for (int64_t m = 0; m < M; ++m) {
      for (int64_t f = 0; f < feat; ++f) acc[f] = mode == 3 ? -INFINITY : 0.0;
      for (int64_t j = 0; j < k; ++j) {
        const float* t = table + idx[m * ldi + j] * ldt;
        if (mode == 3) {
          for (int64_t f = 0; f < feat; ++f) {
            const double v = (double)t[f];
            if (v != v || v > acc[f]) acc[f] = (acc[f] != acc[f]) ? acc[f] : v;
          }
        } else {
          for (int64_t f = 0; f < feat; ++f) acc[f] += (double)t[f];
        }
      }
      for (int64_t f = 0; f < feat; ++f)
        out[m * ldo + f] = (float)(mode == 0 ? acc[f] / (double)k : acc[f]);
    }
    free(acc);
  }
}
