// ORACLE / TEST INFRASTRUCTURE ONLY: the FLOP-counting build of drc_oracle.c
// (see flopcount.hpp).  Same C-ABI as libdrc_oracle.so plus the counters.
#include "flopcount.hpp"
std::atomic<unsigned long long> g_flops{0}, g_flops_nz{0}, g_trans{0};
extern "C" {
#include "drc_oracle.c"
void oracle_flop_counts(unsigned long long* flops, unsigned long long* trans, int reset) {
  *flops = reset ? g_flops.exchange(0) : g_flops.load();
  *trans = reset ? g_trans.exchange(0) : g_trans.load();
  if (reset) g_flops_nz.store(0);
}
/* the nonzero-operand count (flopcount.hpp) since the last reset of either */
void oracle_flop_counts_nz(unsigned long long* flops_nz, int reset) {
  *flops_nz = reset ? g_flops_nz.exchange(0) : g_flops_nz.load();
}
}
