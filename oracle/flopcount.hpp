// ORACLE / TEST INFRASTRUCTURE ONLY.  Counting build of the C restatement
// (oracle/count_build.cpp -> libdrc_oracle_count.so): every `double` of
// drc_oracle.c becomes `Real`, a double whose arithmetic increments a
// process-wide counter -- the algorithmic FP64 operation count of the scalar
// algorithm the kernels run, for bench.py's roofline.
// Counted: + - * / and unary minus 1 each, sqrt 1; fabs / fmin / fmax and
// comparisons 0 (sign / select operations); sin, cos, atan2, acos count
// separately as transcendental calls.  A second counter (g_flops_nz) counts
// only the operations whose operands are all nonzero (a quotient: a nonzero
// numerator): the dense restatement's work on structural zeros -- zero blocks
// of P and A, the identity bound rows, zero-padded vectors -- drops out, which
// is the work a sparse solver (OSQP's CSC KKT) does on the same problem.
#pragma once
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include <atomic>
// process-wide (the batch entry points run their instances on pthreads);
// relaxed increments: only the totals matter
extern std::atomic<unsigned long long> g_flops, g_flops_nz, g_trans;
// one operation; `nz`: its operands are all nonzero
inline void drc_count(bool nz) {
  g_flops.fetch_add(1, std::memory_order_relaxed);
  if (nz) g_flops_nz.fetch_add(1, std::memory_order_relaxed);
}
struct Real {
  double v;
  Real() = default;
  constexpr Real(double x) : v(x) {}
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  Real& operator+=(Real o) { drc_count(v != 0 && o.v != 0); v += o.v; return *this; }
  Real& operator-=(Real o) { drc_count(v != 0 && o.v != 0); v -= o.v; return *this; }
  Real& operator*=(Real o) { drc_count(v != 0 && o.v != 0); v *= o.v; return *this; }
  Real& operator/=(Real o) { drc_count(v != 0); v /= o.v; return *this; }
};
static_assert(sizeof(Real) == 8 && std::is_trivially_copyable<Real>::value, "Real must keep double's layout");
template <class T>
using Arith = typename std::enable_if<std::is_arithmetic<T>::value, Real>::type;
// NZ(a, b): the nonzero-operand rule of the operator (quotients: numerator only)
#define DRC_COUNT_OP(op, NZ)                                                                                     \
  inline Real operator op(Real a, Real b) { drc_count(NZ(a.v, b.v)); return Real(a.v op b.v); }                  \
  template <class T> inline Arith<T> operator op(Real a, T b) { drc_count(NZ(a.v, (double)b)); return Real(a.v op (double)b); } \
  template <class T> inline Arith<T> operator op(T a, Real b) { drc_count(NZ((double)a, b.v)); return Real((double)a op b.v); }
#define DRC_NZ2(x, y) ((x) != 0 && (y) != 0)
#define DRC_NZ1(x, y) ((x) != 0)
DRC_COUNT_OP(+, DRC_NZ2)
DRC_COUNT_OP(-, DRC_NZ2)
DRC_COUNT_OP(*, DRC_NZ2)
DRC_COUNT_OP(/, DRC_NZ1)
#undef DRC_COUNT_OP
inline Real operator-(Real a) { drc_count(a.v != 0); return Real(-a.v); }
inline Real operator+(Real a) { return a; }
#define DRC_COUNT_CMP(op)                                                               \
  inline bool operator op(Real a, Real b) { return a.v op b.v; }                        \
  template <class T> inline typename std::enable_if<std::is_arithmetic<T>::value, bool>::type operator op(Real a, T b) { return a.v op (double)b; } \
  template <class T> inline typename std::enable_if<std::is_arithmetic<T>::value, bool>::type operator op(T a, Real b) { return (double)a op b.v; }
DRC_COUNT_CMP(<)
DRC_COUNT_CMP(>)
DRC_COUNT_CMP(<=)
DRC_COUNT_CMP(>=)
DRC_COUNT_CMP(==)
DRC_COUNT_CMP(!=)
#undef DRC_COUNT_CMP
inline Real sqrt(Real a) { drc_count(a.v != 0); return Real(::sqrt(a.v)); }
inline Real fabs(Real a) { return Real(::fabs(a.v)); }
inline Real fmin(Real a, Real b) { return Real(::fmin(a.v, b.v)); }
inline Real fmax(Real a, Real b) { return Real(::fmax(a.v, b.v)); }
inline Real cos(Real a) { g_trans.fetch_add(1, std::memory_order_relaxed); return Real(::cos(a.v)); }
inline Real sin(Real a) { g_trans.fetch_add(1, std::memory_order_relaxed); return Real(::sin(a.v)); }
inline Real acos(Real a) { g_trans.fetch_add(1, std::memory_order_relaxed); return Real(::acos(a.v)); }
inline Real atan2(Real a, Real b) { g_trans.fetch_add(1, std::memory_order_relaxed); return Real(::atan2(a.v, b.v)); }
inline bool isfinite(Real a) { return std::isfinite(a.v); }
inline bool isnan(Real a) { return std::isnan(a.v); }
#define double Real
