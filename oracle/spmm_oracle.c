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

/* One 32-bit hash of (seed, edge, head): the dropout stream the HIP GAT kernels draw
 * (csrc/gat.hip hash3), restated so that the checker re-derives the training masks. An edge is
 * kept when (h >> 8) / 2^24 >= p, and a kept weight is scaled by 1 / (1 - p) (F.dropout's
 * inverted dropout, where layers.py:30 / :115 apply it). */
static uint32_t oracle_hash3(uint64_t seed, int64_t edge, int64_t head) {
  uint32_t h = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27d4eb2fu);
  h ^= (uint32_t)edge * 0x9e3779b9u;
  h ^= (uint32_t)((uint64_t)edge >> 32) * 0x85ebca6bu;
  h ^= (uint32_t)head * 0xc2b2ae35u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

/* The same hash over (seed, a[i], b[i]) for i < n: the element dropout of a GCN layer trained
 * with its ReLU and Dropout (GCN/GCN.py:12-14) in the transform epilogue (csrc/common.hpp
 * dropout_hash over (row, column)); keep[i] = 1 iff (h >> 8) / 2^24 >= p. */
void oracle_dropout_keep(uint64_t seed, const int64_t* a, const int64_t* b, int64_t n, float p,
                         uint8_t* keep) {
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t h = oracle_hash3(seed, a[i], b[i]);
        keep[i] = (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
    }
}

/*
 * Forward + backward of the H-head attention block of GATBase (GAT/models/GAT.py:16, each head
 * GAT/models/layers.py:22-37 dense or :94-131 sparse, concat=True: ELU applied) in float64,
 * given Wh = X W (double [n, H fh]) and the loss gradient gy (float [n, H fh]):
 *   el_i = a_src . Wh_i, er_j = a_dst . Wh_j (per head), t_ij = el_i + er_j,
 *   z_ij = LeakyReLU(t_ij) (dense) or -LeakyReLU(t_ij) (sparse), a_ij = softmax_j z_ij,
 *   w_ij = a_ij m_ij (m_ij = 0 or 1 / (1 - p), the dropout mask), pre_i = sum_j w_ij Wh_j,
 *   out_i = ELU(pre_i)  (if elu);
 *   dout_i = gy_i ELU'(pre_i), g_ij = dout_i . Wh_j, D_i = sum_j w_ij g_ij,
 *   dz_ij = a_ij (m_ij g_ij - D_i), dt_ij = +-dz_ij LeakyReLU'(t_ij),
 *   del_i = sum_j dt_ij, der_j = sum_i dt_ij,
 *   dWh_j = sum_i w_ij dout_i + der_j a_dst + del_j a_src.
 * The autograd of the reference's layer (SpecialSpmmFunction.backward, layers.py:54-64, for the
 * sparse one). Row-parallel first pass (per-edge w_ij and dt_ij kept), then a column-parallel
 * pass over the transposed edge order: deterministic, no atomics. Every row must have an edge
 * (the GCN-normalised graphs carry self-loops). Returns 0, or -1 if a row is edgeless / -2 if
 * memory runs out.
 * kink_del / kink_der (nullable): LeakyReLU' jumps from 1 to slope at t = 0, so an edge whose
 * t_ij lies within fp32 rounding of 0 (|t| <= 1e-5 (|a_src| . |Wh_i| + |a_dst| . |Wh_j|)) may take
 * either branch in an fp32 implementation; its |dz_ij| (1 - slope) is summed per row into
 * kink_del and per column into kink_der: the slack a checker allows those rows. wh_abs
 * (nullable: |wh|) is the magnitude Wh was summed from (|X| |W|), the scale of its rounding.
 */
int oracle_gat_block_grad(const int64_t* rowptr, const int32_t* col, int64_t n,
                          const double* wh, const double* wh_abs, const float* a_src, const float* a_dst,
                          const float* gy, int64_t heads, int64_t fh, double slope, int sparse,
                          int elu, double drop_p, uint64_t drop_seed, double* out, double* dwh,
                          double* del, double* der, double* kink_del, double* kink_der) {
  const int64_t F = heads * fh, nnz = rowptr[n];
  for (int64_t r = 0; r < n; ++r)
    if (rowptr[r + 1] == rowptr[r]) return -1;
  double* el = (double*)malloc(sizeof(double) * (size_t)(n * heads));
  double* er = (double*)malloc(sizeof(double) * (size_t)(n * heads));
  double* ela = (double*)malloc(sizeof(double) * (size_t)(n * heads));
  double* era = (double*)malloc(sizeof(double) * (size_t)(n * heads));
  double* kk = (double*)calloc((size_t)(nnz * heads > 0 ? nnz * heads : 1), sizeof(double));
  double* dout = (double*)malloc(sizeof(double) * (size_t)(n * F));
  double* w = (double*)malloc(sizeof(double) * (size_t)(nnz * heads));
  double* dt = (double*)malloc(sizeof(double) * (size_t)(nnz * heads));
  int64_t* cptr = (int64_t*)calloc((size_t)(n + 1), sizeof(int64_t));
  int64_t* perm = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nnz > 0 ? nnz : 1));
  int64_t* rowof = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nnz > 0 ? nnz : 1));
  if (!el || !er || !ela || !era || !kk || !dout || !w || !dt || !cptr || !perm || !rowof) {
    free(el); free(er); free(ela); free(era); free(kk); free(dout); free(w); free(dt);
    free(cptr); free(perm); free(rowof);
    return -2;
  }
  const double scale = drop_p > 0 ? 1.0 / (1.0 - drop_p) : 1.0;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i)
    for (int64_t h = 0; h < heads; ++h) {
      double s = 0, d = 0, sa = 0, da = 0;
      for (int64_t f = 0; f < fh; ++f) {
        const double x = wh[i * F + h * fh + f];
        const double xa = wh_abs ? wh_abs[i * F + h * fh + f] : fabs(x);
        s += (double)a_src[h * fh + f] * x;
        d += (double)a_dst[h * fh + f] * x;
        sa += fabs((double)a_src[h * fh + f]) * xa;
        da += fabs((double)a_dst[h * fh + f]) * xa;
      }
      el[i * heads + h] = s;
      er[i * heads + h] = d;
      ela[i * heads + h] = sa;
      era[i * heads + h] = da;
    }
#pragma omp parallel
  {
    double* pre = (double*)malloc(sizeof(double) * (size_t)F);
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t e0 = rowptr[i], e1 = rowptr[i + 1];
      for (int64_t e = e0; e < e1; ++e) rowof[e] = i;
      for (int64_t h = 0; h < heads; ++h) {
        double mx = -INFINITY, l = 0;
        for (int64_t e = e0; e < e1; ++e) {
          double t = el[i * heads + h] + er[(int64_t)col[e] * heads + h];
          double z = t > 0 ? t : slope * t;
          if (sparse) z = -z;
          dt[e * heads + h] = z;  /* z for now */
          if (z > mx) mx = z;
        }
        if (sparse) mx = 0;  /* the reference's exp(-LeakyReLU) has no max shift */
        for (int64_t e = e0; e < e1; ++e) l += exp(dt[e * heads + h] - mx);
        for (int64_t f = 0; f < fh; ++f) pre[h * fh + f] = 0;
        for (int64_t e = e0; e < e1; ++e) {
          const double a = exp(dt[e * heads + h] - mx) / l;
          double m = 1.0;
          if (drop_p > 0) {
            const uint32_t r = oracle_hash3(drop_seed, e, h);
            m = ((double)(r >> 8) * (1.0 / 16777216.0) < drop_p) ? 0.0 : scale;
          }
          dt[e * heads + h] = a;  /* a for now */
          w[e * heads + h] = a * m;
          const double* x = wh + (int64_t)col[e] * F + h * fh;
          for (int64_t f = 0; f < fh; ++f) pre[h * fh + f] += a * m * x[f];
        }
      }
      for (int64_t f = 0; f < F; ++f) {
        const double p = pre[f];
        out[i * F + f] = elu ? (p > 0 ? p : expm1(p)) : p;
        dout[i * F + f] = (double)gy[i * F + f] * (elu ? (p > 0 ? 1.0 : exp(p)) : 1.0);
      }
      for (int64_t h = 0; h < heads; ++h) {
        double D = 0;
        for (int64_t f = 0; f < fh; ++f) D += dout[i * F + h * fh + f] * pre[h * fh + f];
        double dl = 0, kdl = 0;
        for (int64_t e = e0; e < e1; ++e) {
          const double* x = wh + (int64_t)col[e] * F + h * fh;
          double g = 0;
          for (int64_t f = 0; f < fh; ++f) g += dout[i * F + h * fh + f] * x[f];
          const double a = dt[e * heads + h];
          double m = 1.0;
          if (drop_p > 0) {
            const uint32_t r = oracle_hash3(drop_seed, e, h);
            m = ((double)(r >> 8) * (1.0 / 16777216.0) < drop_p) ? 0.0 : scale;
          }
          const double dz = a * (m * g - D);
          const double t = el[i * heads + h] + er[(int64_t)col[e] * heads + h];
          const double v = (sparse ? -dz : dz) * (t > 0 ? 1.0 : slope);
          dt[e * heads + h] = v;
          dl += v;
          if (fabs(t) <= 1e-5 * (ela[i * heads + h] + era[(int64_t)col[e] * heads + h])) {
            kk[e * heads + h] = fabs(dz) * (1.0 - slope);
            kdl += kk[e * heads + h];
          }
        }
        del[i * heads + h] = dl;
        if (kink_del) kink_del[i * heads + h] = kdl;
      }
    }
    free(pre);
  }
  /* transposed edge order: counting sort by column (stable: rows ascending per column) */
  for (int64_t e = 0; e < nnz; ++e) cptr[col[e] + 1]++;
  for (int64_t j = 0; j < n; ++j) cptr[j + 1] += cptr[j];
  {
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t j = 0; j < n; ++j) fill[j] = cptr[j];
    for (int64_t e = 0; e < nnz; ++e) perm[fill[col[e]]++] = e;
    free(fill);
  }
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t j = 0; j < n; ++j) {
    double* dj = dwh + j * F;
    for (int64_t f = 0; f < F; ++f) dj[f] = 0;
    for (int64_t h = 0; h < heads; ++h) {
      der[j * heads + h] = 0;
      if (kink_der) kink_der[j * heads + h] = 0;
    }
    for (int64_t q = cptr[j]; q < cptr[j + 1]; ++q) {
      const int64_t e = perm[q], i = rowof[e];
      for (int64_t h = 0; h < heads; ++h) {
        const double ww = w[e * heads + h];
        der[j * heads + h] += dt[e * heads + h];
        if (kink_der) kink_der[j * heads + h] += kk[e * heads + h];
        for (int64_t f = 0; f < fh; ++f) dj[h * fh + f] += ww * dout[i * F + h * fh + f];
      }
    }
    for (int64_t h = 0; h < heads; ++h)
      for (int64_t f = 0; f < fh; ++f)
        dj[h * fh + f] += der[j * heads + h] * (double)a_dst[h * fh + f] +
                          del[j * heads + h] * (double)a_src[h * fh + f];
  }
  free(el); free(er); free(ela); free(era); free(kk); free(dout); free(w); free(dt);
  free(cptr); free(perm); free(rowof);
  return 0;
}
