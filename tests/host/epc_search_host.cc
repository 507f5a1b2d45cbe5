// Host build of the EPC multiplier search (admm-quantization_amd/csrc/epc_search.h, the state
// machine both device forms of cp_anc's mode update run) for CPU tests: e(mu) from an
// eigen-form spectrum, the search driven to completion. Test infrastructure only
// (tests/test_epc_search_host.py builds it with g++; nothing here ships).
#include <cmath>
#define __host__
#define __device__
#include "../../admm-quantization_amd/csrc/epc_search.h"

using namespace admmq;

extern "C" int epc_search_run(const double* c, const double* s, int n, double normY2, double delta2, double warm,
                              double tr, double fail_below, double* mu_out, int* evals_out) {
  EpcSearch st;
  epc_search_init(st, warm);
  int evals = 0;
  for (int guard = 0; guard < 400; ++guard) {
    epc_search_next(st, warm, tr, delta2);
    if (st.state == EPC_DONE) break;
    const double at = st.at;
    ++evals;
    // a factorisation of G + at I fails below `fail_below` (an indefinite G's smallest eigenvalue)
    const bool ok = at > fail_below;
    double f = 0.0, g = 0.0, h = 0.0;
    if (ok)
      for (int i = 0; i < n; ++i) {
        const double d = s[i] + at;
        f += c[i] / d;
        g += c[i] / (d * d);
        h += c[i] / (d * d * d);
      }
    epc_search_absorb(st, ok, normY2 - f - at * g, 2.0 * at * h, h, delta2, normY2);
  }
  *mu_out = st.mu;
  *evals_out = evals;
  return epc_search_ok(st) ? 0 : 1;
}
