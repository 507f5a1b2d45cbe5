// The EPC step's multiplier search (musco cp_anc's mode update, source/parafac_epc.py:61-74):
// mu >= 0 with e(mu) = ||Y||^2 - <F, X> - mu ||X||^2 = delta^2, X = F (G + mu I)^-1, by
// safeguarded Newton steps on e (e' = 2 mu <X, X (G + mu I)^-1>) inside a bracket [lo, hi].
// One state machine shared by the two forms of the step:
//   * k_epc_step64 (epc_kernels.hip, n <= 136): thread 0 of the one workgroup decides between
//     evaluations, the state in LDS;
//   * the blocked step (solve64.hip, any n): a one-thread kernel after every evaluation round
//     (Cholesky of G + mu I, three fp64 products, their sums), the state in global memory.
// States:
//   WARM   the warm start, when > 0: e < delta2 puts the root above it (mu > 0 for sure),
//          otherwise Newton steps go down from it inside [0, warm];
//   ZERO   mu = 0 (first, without a warm start; else when a Newton step from above leaves
//          the bracket): e(0) >= delta2 means the LS step keeps the error (mu = 0, done);
//   GROW   no upper end yet: from max(lo, trace / n 2^-20), doubling / Newton steps;
//   NEWTON safeguarded Newton inside [lo, hi] until the step is below kEpcMuTol, the bracket
//          has collapsed or e is at its rounding floor (e is flat near mu = 0, e'(0) = 0, so
//          a small |e - delta2| alone does not fix mu: the step decides). A point reached by
//          a Newton step of relative size <= kEpcMuQuad is accepted without evaluating the
//          next step: Newton converges quadratically, so that step would be ~kEpcMuQuad^2
//          (the confirming evaluation was a third of a warm-started step's evaluations).
// A failed factorisation at mu (G + mu I not numerically positive definite) only raises lo.
#pragma once

namespace admmq {

// mu to 1e-12 relative: X = F (G + mu I)^-1 moves by at most mu_err / (lambda_min + mu) <= 1e-12
// relative (mu itself is ill-determined where e is flat, e'(0) = 0: there only X matters)
constexpr double kEpcMuTol = 1e-12;
constexpr double kEpcMuQuad = 1e-6;   // sqrt(kEpcMuTol)

enum { EPC_WARM = 0, EPC_ZERO, EPC_GROW, EPC_NEWTON, EPC_DONE, EPC_FINAL };

// pmu: the mu of the last successful evaluation (NaN after a failed one)
// lastrel: the relative size of the Newton step that chose `at` (infinite for other choices)
struct EpcSearch { double e, de, mu, lo, hi, at, pmu, q0, lastrel; int state, have, need0, pad_; };

__host__ __device__ inline void epc_search_init(EpcSearch& st, double warm) {
  st.e = st.de = st.mu = st.lo = 0.0;
  st.hi = __builtin_huge_val();
  st.pmu = __builtin_nan("");
  st.q0 = 0.0;
  st.at = 0.0;
  st.lastrel = __builtin_huge_val();
  st.state = warm > 0.0 ? EPC_WARM : EPC_ZERO;
  st.have = 0;
  st.need0 = 1;
  st.pad_ = 0;
}

// Where to evaluate next (st.at), or st.state = EPC_DONE. tr: trace(G) / n.
__host__ __device__ inline void epc_search_next(EpcSearch& st, double warm, double tr, double delta2) {
  for (;;) {
    const int state = st.state;
    if (state == EPC_WARM) { st.at = warm; return; }
    if (state == EPC_ZERO) { st.at = 0.0; return; }
    // the point just evaluated came from a Newton step of relative size <= kEpcMuQuad (and
    // was factorised): accept it
    if (st.lastrel <= kEpcMuQuad && st.pmu == st.mu && st.pmu == st.at) { st.state = EPC_DONE; return; }
    st.lastrel = __builtin_huge_val();
    if (state == EPC_GROW) {
      double at = st.have ? 2.0 * fmax(st.mu, st.lo) : (st.q0 > 0.0 ? st.q0 : (tr > 0.0 ? tr * 0x1p-20 : 1e-300));
      // no successful evaluation yet but failed ones: a shift too small to factor, so the next
      // one is at least twice the largest failed shift (never the same mu again)
      if (!st.have && st.lo > 0.0) at = fmax(at, 2.0 * st.lo);
      if (st.have && st.de > 0.0) {   // a Newton step from below (lands above the root: e convex near it)
        const double nx = st.mu - (st.e - delta2) / st.de;
        if (fabs(nx - st.mu) <= kEpcMuTol * st.mu) { st.state = EPC_DONE; return; }   // converged from below
        if (nx > st.mu && nx < at) { at = nx; st.lastrel = (nx - st.mu) / st.mu; }
      }
      if (!(at < 1e300)) { st.state = EPC_DONE; return; }
      st.at = at;
      return;
    }
    if (state == EPC_NEWTON) {
      if (!(st.hi - st.lo > kEpcMuTol * st.hi)) { st.state = EPC_DONE; return; }   // collapsed bracket
      double nx = st.de > 0.0 ? st.mu - (st.e - delta2) / st.de : -1.0;
      if (!(nx > st.lo && nx < st.hi) && st.need0) { st.state = EPC_ZERO; continue; }   // below the bracket: is mu = 0 the answer?
      const bool newton = nx > st.lo && nx < st.hi;
      if (!newton) nx = 0.5 * (st.lo + st.hi);
      if (fabs(nx - st.mu) <= kEpcMuTol * st.mu) { st.state = EPC_DONE; return; }   // converged
      if (newton && st.mu > 0.0) st.lastrel = fabs(nx - st.mu) / st.mu;
      st.at = nx;
      return;
    }
    return;   // DONE
  }
}

// Takes the evaluation at st.at: ok (the factorisation succeeded), en = e(at), dn = e'(at),
// h = <X, X (G + at I)^-1> (the cold start's model curvature).
__host__ __device__ inline void epc_search_absorb(EpcSearch& st, bool ok, double en, double dn, double h,
                                                  double delta2, double normY2) {
  const double at = st.at;
  st.pmu = ok ? at : __builtin_nan("");
  const int state = st.state;
  if (state == EPC_WARM) {
    // above the root: Newton down from the warm start, e(0) only if a step leaves the
    // bracket (the LS step may keep the error: mu = 0); below it: grow
    if (ok) {
      st.mu = at; st.e = en; st.de = dn; st.have = 1;
      if (en < delta2) { st.lo = at; st.need0 = 0; }
      else st.hi = at;
    }
    st.state = !ok ? EPC_ZERO : (st.need0 ? EPC_NEWTON : EPC_GROW);
  } else if (state == EPC_ZERO) {
    if (ok && en >= delta2) { st.mu = 0.0; st.have = 0; st.state = EPC_DONE; }   // the LS step: mu = 0
    else {
      // a cold start's first step from the model e(mu) ~ e(0) + mu^2 <X0, X0 G^-1> near 0:
      // it lands at or below the root where <X, X A^-1> falls with mu, so the growth
      // continues from there
      if (ok && h > 0.0) st.q0 = sqrt((delta2 - en) / h);
      st.need0 = 0;
      st.state = (st.have && st.hi < __builtin_huge_val()) ? EPC_NEWTON : EPC_GROW;
    }
  } else if (state == EPC_GROW) {
    if (!ok) st.lo = fmax(st.lo, at);
    else {
      st.mu = at; st.e = en; st.de = dn; st.have = 1;
      if (en < delta2) st.lo = at;
      else { st.hi = at; st.state = EPC_NEWTON; }
    }
  } else if (state == EPC_NEWTON) {
    if (!ok) st.lo = fmax(st.lo, at);
    else {
      st.mu = at; st.e = en; st.de = dn;
      if (en < delta2) { st.lo = at; st.need0 = 0; } else st.hi = at;   // (e increases with mu: e(0) <= e(lo))
      if (fabs(en - delta2) <= 16.0 * 0x1p-52 * normY2) st.state = EPC_DONE;   // at the rounding floor of e
    }
  }
}

// The step's result is valid when the last successful evaluation is at the returned mu
// (or mu = 0 was accepted from e(0)).
__host__ __device__ inline bool epc_search_ok(const EpcSearch& st) {
  return st.state == EPC_DONE && st.pmu == st.mu && (st.have || st.mu == 0.0);
}

}  // namespace admmq
