// Host side of the MI355X-native QP-IK: the C-ABI of include/drc_amd.h.
// Model build and upload, per-stream scratch, the launch sequences (task ->
// QP kernels on forked sub-batch streams, QPID, closed-form controllers), the
// synchronous host-buffer entries and the dynamics entries.  The kernels live
// in task_kernel.hip, qp_kernel.hip, qpid_kernel.hip and dynamics.hip.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/drc_amd.h"
#include "../../include/drc_amd_debug.h"
#include "dynamics.hpp"
#include "kernel_common.hpp"
#include "launch.hpp"

// ==========================================================================
// host side: the C-ABI (include/drc_amd.h)
// ==========================================================================
namespace drc_amd {

// Per-stream scratch of a model: the task-record pool, the work-queue
// counters and the COD list.  Calls on one stream are ordered by that stream,
// so they may share it; calls on two streams get disjoint contexts (the
// C-ABI's "reentrant per stream", include/drc_amd.h).  At most kMaxStreamCtx
// contexts are kept: a new stream beyond that evicts the least recently used
// one (once the last call that used it has finished: `done`, an event recorded
// on the caller's stream after each call's launches), and
// drc_model_release_stream frees a stream's context at once, so a caller
// cycling through streams holds a bounded amount of device memory.
struct StreamCtx {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // recorded on `stream` after every call's launches
  uint64_t last_use = 0;
  void* pool = nullptr;  // task records / QPID dynamics / OSF M^-1, g
  int64_t pool_bytes = 0;
  // work-queue counters: [slot][kernel (task, QP)][8 XCD classes]; slots
  // 0..15 the QPIK sub-batches, 16 QPID, 17 the closed-form controllers
  static constexpr int kSlotInts = 32;  // task queue 8, QP queue 8, lane-stage hard count 1
  static constexpr int kQueueSlotQpid = 16, kQueueSlotCf = 17, kQueueInts = 18 * kSlotInts;
  int* d_queue = nullptr;
  int* dyn_list = nullptr;  // instances whose M_inv needs the serial COD
  int64_t dyn_list_cap = 0;
};
constexpr size_t kMaxStreamCtx = 8;

// Fork/join streams of the concurrent sub-batches, shared by every caller
// stream of a model: a process gets 4 hardware queues (GPU_MAX_HW_QUEUES), so
// the internal streams do not multiply with the caller's streams.  Calls are
// enqueued under the model's launch mutex, so an event is recorded and waited
// on by one call before the next re-records it; work of two caller streams on
// one lane runs in order (each call on its own context's scratch).
struct Lanes {
  std::vector<hipStream_t> lanes;  // concurrent sub-batches (drc_set_concurrency)
  std::vector<hipEvent_t> joins;
  // per sub-batch: the lane stage's hard instances run their task kernel on a
  // side stream while the QP of the other instances runs
  std::vector<hipStream_t> sides;
  std::vector<hipEvent_t> side_fork, side_join;
  hipEvent_t fork = nullptr;
};

struct drc_model_impl {
  HostModel hm;
  DevModel* d_model = nullptr;
  int device = 0;
  drc_kinematic_param kparam{};
  drc_joint_index jidx{};
  drc_actuator_index aidx{};
  std::vector<std::unique_ptr<StreamCtx>> ctxs;  // one per caller stream seen (at most kMaxStreamCtx)
  uint64_t ctx_tick = 0;
  Lanes ln;
  int timing = 0;  // drc_debug_kernel_timing: HIP events around each launch
  int lane_stage = 0;  // drc_debug_lane_stage: 0 off, 1 lane stage + side-stream hard path, 2 + serial hard path, 3 auto
  // timed calls: {caller-stream start, caller-stream end, per chunk: task start, task end, qp end}
  // timed calls: {call start, call end, task start, task end, QP end of the
  // sub-batch on the caller's stream} and the call's sub-batch count
  std::vector<std::pair<std::vector<hipEvent_t>, int>> events;
  std::vector<hipEvent_t> evpool;  // timing events returned by drc_debug_kernel_times, reused
  // concurrent sub-batches: the batch is cut into `chunks` contiguous ranges,
  // the last on the caller's stream and the others on internal streams forked
  // from / joined to it, so one range's task kernel overlaps another's QP
  // kernel and the straggler tails of the kernels interleave.  4 streams fit
  // the 4 hardware queues a process gets by default; measured on MI355X
  // (r04u, B = 65 536): 4 sub-batches FR3 23.6 M / UR5e 20.3 M / XLS-FR3 17.9 M
  // against 22.6 / 19.1 / 17.7 M at 3 (then on 3 internal streams + the
  // caller's); 6 sub-batches, with 8 hardware queues or 4, were slower
  int chunks = 4;
  // fused task + QP kernel for the compiled QPIK shapes and small batches
  // (fused_kernel.hip; drc_set_fusion): one launch per call, the record in LDS
  int fused = 1;
  // drc_debug_instance_order: a scheduling order for calls of exactly
  // order_n instances (device copy), or none
  int32_t* d_order = nullptr;
  int64_t order_n = 0;
  // host-buffer entry points: device staging + an internal stream
  std::mutex host_mu;
  void* stage = nullptr;
  int64_t stage_bytes = 0;
  // pinned host mirror of the staging buffer: the synchronous entries pack
  // their inputs into it and copy them over in one transfer, and bring the
  // outputs back in one (drc_qpik_host, drc_state_host: B = 1 control cycles)
  double* pinned = nullptr;
  int64_t pinned_bytes = 0;
  hipStream_t hstream = nullptr;
  hipEvent_t hdone = nullptr;  // recorded after a synchronous entry's copy back
  // drc_debug_host_timeline: per synchronous call, steady-clock ns at entry,
  // inputs packed, H2D + launches + D2H enqueued, completion seen, exit
  int tl_on = 0;
  std::vector<int64_t> tl;
  std::mutex mu;         // the context list, timing events, concurrency
  std::mutex launch_mu;  // one call's launch sequence is enqueued as a unit, so
                         // two host threads sharing a stream cannot interleave
                         // their kernels on its scratch
};

static thread_local std::string g_last_error;
static int set_err(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return set_err(DRC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void free_ctx(StreamCtx* c) {
  // the event outlives a destroyed stream: waiting on it orders the frees
  // after this context's last use without draining any other stream
  if (c->done) (void)hipEventSynchronize(c->done), (void)hipEventDestroy(c->done);
  c->done = nullptr;
  if (c->d_queue) (void)hipFree(c->d_queue);
  if (c->pool) (void)hipFree(c->pool);
  if (c->dyn_list) (void)hipFree(c->dyn_list);
  c->d_queue = nullptr;
  c->pool = nullptr;
  c->dyn_list = nullptr;
}

// Records a stream context's `done` event on every exit of a launch path
// once the context is in use, so eviction (free_ctx) never frees scratch that
// kernels of this call still use.  Every launch path enqueues on the caller's
// stream only, except the QPIK path's concurrent sub-batches: a call that
// fails after forking may have left kernels on the model's internal fork /
// side streams that `done` on the caller's stream does not follow, so that
// path (forks set) waits for those streams -- the model's own, never the
// device: other streams and models in the process are not stalled, and a
// failure before anything was forked costs no synchronisation at all.
struct DoneGuard {
  StreamCtx* const& cx;
  hipStream_t st;
  const Lanes* forks = nullptr;  // set once a sub-batch may run on a fork stream
  bool ok = false;
  ~DoneGuard() {
    if (!cx || !cx->done) return;
    if (!ok && forks) {
      for (hipStream_t s : forks->lanes) (void)hipStreamSynchronize(s);
      for (hipStream_t s : forks->sides) (void)hipStreamSynchronize(s);
    }
    (void)hipEventRecord(cx->done, st);
  }
};

// A tuning knob from the environment: its integer value when set and
// parsable, clamped to >= lo; otherwise the default.
static int64_t env_int(const char* name, int64_t def, int64_t lo) {
  const char* v = getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  const long long x = strtoll(v, &end, 10);
  if (end == v) return def;
  return x < lo ? lo : x;
}

// The scratch context of `st` (created on first use; the caller holds
// m->launch_mu and m->mu, so no launch still being enqueued uses an evicted
// context).  Beyond kMaxStreamCtx streams the least recently used context is
// freed once its `done` event has completed (its stream may already be
// destroyed; the event stays valid, and no other stream is waited for).
static int stream_ctx(drc_model_impl* m, hipStream_t st, StreamCtx** out) {
  for (auto& c : m->ctxs)
    if (c->stream == st) {
      c->last_use = ++m->ctx_tick;
      *out = c.get();
      return DRC_OK;
    }
  if (m->ctxs.size() >= kMaxStreamCtx) {
    size_t lru = 0;
    for (size_t i = 1; i < m->ctxs.size(); ++i)
      if (m->ctxs[i]->last_use < m->ctxs[lru]->last_use) lru = i;
    free_ctx(m->ctxs[lru].get());
    m->ctxs.erase(m->ctxs.begin() + static_cast<std::ptrdiff_t>(lru));
  }
  std::unique_ptr<StreamCtx> c(new StreamCtx());
  c->stream = st;
  c->last_use = ++m->ctx_tick;
  HIP_TRY(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
  HIP_TRY(hipMalloc(&c->d_queue, StreamCtx::kQueueInts * sizeof(int)));
  *out = c.get();
  m->ctxs.push_back(std::move(c));
  return DRC_OK;
}
static int ensure_pool(StreamCtx* c, int64_t bytes) {
  if (c->pool_bytes >= bytes) return DRC_OK;
  if (c->pool) HIP_TRY(hipFree(c->pool));  // synchronises: no launch still reads it
  c->pool = nullptr;
  c->pool_bytes = 0;
  HIP_TRY(hipMalloc(&c->pool, bytes));
  c->pool_bytes = bytes;
  return DRC_OK;
}
static void free_lanes(Lanes* c) {
  for (hipStream_t ls : c->lanes) (void)hipStreamSynchronize(ls);
  for (hipStream_t ls : c->sides) (void)hipStreamSynchronize(ls);
  for (hipStream_t ls : c->lanes) (void)hipStreamDestroy(ls);
  for (hipEvent_t e : c->joins) (void)hipEventDestroy(e);
  for (hipStream_t ls : c->sides) (void)hipStreamDestroy(ls);
  for (hipEvent_t e : c->side_fork) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->side_join) (void)hipEventDestroy(e);
  if (c->fork) (void)hipEventDestroy(c->fork);
}

// DyrosMath::PinvCOD on a small dense matrix (host, model build only):
// Moore-Penrose inverse via the normal equations' symmetric eigen-system,
// rank cut at 1e-6 relative (math_type_define.h:7,563-570).
static void pinv_small(const double* A, int r, int c, double* X /* c x r */) {
  // X = (A^T A)^+ A^T with (A^T A) symmetric c x c (c <= 3 here)
  double N[9] = {0}, V[9], w[3];
  for (int i = 0; i < c; ++i)
    for (int j = 0; j < c; ++j)
      for (int k = 0; k < r; ++k) N[i * c + j] += A[k * c + i] * A[k * c + j];
  for (int i = 0; i < c * c; ++i) V[i] = (i % (c + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int i = 0; i < c; ++i)
      for (int j = i + 1; j < c; ++j) off += N[i * c + j] * N[i * c + j];
    if (off < 1e-300) break;
    for (int p = 0; p < c; ++p)
      for (int q = p + 1; q < c; ++q) {
        if (std::fabs(N[p * c + q]) < 1e-300) continue;
        double th = (N[q * c + q] - N[p * c + p]) / (2 * N[p * c + q]);
        double t = (th >= 0 ? 1 : -1) / (std::fabs(th) + std::sqrt(th * th + 1));
        double cs = 1 / std::sqrt(t * t + 1), sn = t * cs;
        for (int k = 0; k < c; ++k) {
          double a = N[k * c + p], b = N[k * c + q];
          N[k * c + p] = cs * a - sn * b;
          N[k * c + q] = sn * a + cs * b;
        }
        for (int k = 0; k < c; ++k) {
          double a = N[p * c + k], b = N[q * c + k];
          N[p * c + k] = cs * a - sn * b;
          N[q * c + k] = sn * a + cs * b;
        }
        for (int k = 0; k < c; ++k) {
          double a = V[k * c + p], b = V[k * c + q];
          V[k * c + p] = cs * a - sn * b;
          V[k * c + q] = sn * a + cs * b;
        }
      }
  }
  double wmax = 0;
  for (int i = 0; i < c; ++i) {
    w[i] = N[i * c + i];
    wmax = std::fmax(wmax, std::fabs(w[i]));
  }
  double Ni[9] = {0};
  for (int e = 0; e < c; ++e) {
    if (std::sqrt(std::fabs(w[e])) <= 1e-6 * std::sqrt(wmax)) continue;
    for (int i = 0; i < c; ++i)
      for (int j = 0; j < c; ++j) Ni[i * c + j] += V[i * c + e] * V[j * c + e] / w[e];
  }
  for (int i = 0; i < c; ++i)
    for (int k = 0; k < r; ++k) {
      double s = 0;
      for (int j = 0; j < c; ++j) s += Ni[i * c + j] * A[k * c + j];
      X[i * r + k] = s;
    }
}

// Mobile::RobotData::computeFKJacobian (src/mobile/robot_data.cpp:123-204) at
// the wheel positions `wheel_pos` (used by the caster drive only; may be NULL
// for the configuration-independent drives, then zero steer angles).
static int mobile_fk_jacobian(const drc_kinematic_param& p, int* W, double out[3][kMaxWheels],
                              const double* wheel_pos = nullptr) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < kMaxWheels; ++c) out[r][c] = 0;
  if (p.type == DRC_DRIVE_DIFFERENTIAL) {
    *W = 2;
    out[0][0] = p.wheel_radius / 2.;
    out[0][1] = p.wheel_radius / 2.;
    out[2][0] = -p.wheel_radius / p.base_width;
    out[2][1] = p.wheel_radius / p.base_width;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_MECANUM) {
    const int n = p.n_wheels;
    if (n < 1 || n > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "mecanum wheel count out of range");
    double Jinv[kMaxWheels * 3], X[3 * kMaxWheels];
    for (int i = 0; i < n; ++i) {
      const double r = p.wheel_radius, g = p.roller_angles[i], px = p.base2wheel_positions[i][0],
                   py = p.base2wheel_positions[i][1], pt = p.base2wheel_angles[i];
      // (1/r) [1 tan g] [[cos pt, sin pt], [-sin pt, cos pt]] [[1 0 -py], [0 1 px]]
      const double a0 = std::cos(pt) - std::tan(g) * std::sin(pt), a1 = std::sin(pt) + std::tan(g) * std::cos(pt);
      Jinv[i * 3 + 0] = a0 / r;
      Jinv[i * 3 + 1] = a1 / r;
      Jinv[i * 3 + 2] = (-a0 * py + a1 * px) / r;
    }
    pinv_small(Jinv, n, 3, X);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < n; ++c) out[r][c] = X[r * n + c];
    *W = n;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_CASTER) {  // CasterFKJacobian (:179-204): W = 2 x casters
    const int C = p.n_wheels;
    if (C < 1 || 2 * C > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "caster count out of range");
    double zero[kMaxWheels] = {0};
    caster_fk_jacobian(C, p.wheel_radius, p.wheel_offset, p.base2wheel_positions, wheel_pos ? wheel_pos : zero, out);
    *W = 2 * C;
    return DRC_OK;
  }
  return set_err(DRC_ERR_INVALID_ARGUMENT, "unknown drive type");
}

// Mobile::RobotController::computeIKJacobian (src/mobile/robot_controller.cpp:55-125):
// wheel velocities = J_ik (W x 3, row-major) * base twist.
static int mobile_ik_jacobian(const drc_kinematic_param& p, const double* wheel_pos, double* J, int* W) {
  const double r = p.wheel_radius;
  if (p.type == DRC_DRIVE_DIFFERENTIAL) {  // DifferentialIKJacobian (:76-84)
    *W = 2;
    const double e[6] = {1 / r, 0, -p.base_width / (2 * r), 1 / r, 0, p.base_width / (2 * r)};
    for (int i = 0; i < 6; ++i) J[i] = e[i];
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_MECANUM) {  // MecanumIKJacobian (:86-107)
    const int n = p.n_wheels;
    if (n < 1 || n > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "mecanum wheel count out of range");
    for (int i = 0; i < n; ++i) {
      const double g = p.roller_angles[i], px = p.base2wheel_positions[i][0], py = p.base2wheel_positions[i][1],
                   pt = p.base2wheel_angles[i];
      const double a0 = std::cos(pt) - std::tan(g) * std::sin(pt), a1 = std::sin(pt) + std::tan(g) * std::cos(pt);
      J[i * 3 + 0] = a0 / r;
      J[i * 3 + 1] = a1 / r;
      J[i * 3 + 2] = (-a0 * py + a1 * px) / r;
    }
    *W = n;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_CASTER) {  // CasterIKJacobian (:109-125), steer angle = wheel_pos(2i)
    const int C = p.n_wheels;
    if (C < 1 || 2 * C > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "caster count out of range");
    const double b = p.wheel_offset;
    for (int i = 0; i < C; ++i) {
      const double phi = wheel_pos ? wheel_pos[2 * i] : 0.0, sp = std::sin(phi), cp = std::cos(phi);
      const double px = p.base2wheel_positions[i][0], py = p.base2wheel_positions[i][1];
      double* r0 = J + (2 * i) * 3;
      double* r1 = J + (2 * i + 1) * 3;
      r0[0] = -sp / b;
      r0[1] = cp / b;
      r0[2] = (px * cp + py * sp) / b - 1;
      r1[0] = cp / r;
      r1[1] = sp / r;
      r1[2] = (px * sp - py * cp) / r;
    }
    *W = 2 * C;
    return DRC_OK;
  }
  return set_err(DRC_ERR_INVALID_ARGUMENT, "unknown drive type");
}

static int upload(drc_model_impl* m) {
  HIP_TRY(hipSetDevice(m->device));
  HIP_TRY(hipMalloc(&m->d_model, sizeof(DevModel)));
  HIP_TRY(hipMemcpy(m->d_model, &m->hm.dev, sizeof(DevModel), hipMemcpyHostToDevice));
  return DRC_OK;
}

// LDS plan: persistent QP region + a union of (kinematics | K^-1 | polish).
// Lanes per QP instance: kQpGroup (kernel_common.hpp); 32 packs two instances
// per wave (Grp<32>: group reductions, DPP / ds_bpermute broadcasts,
// per-group instance sequence and LDS plan; parity tests green) but measured
// slower on FR3: 13.7 M solves/s at two waves per SIMD, 13.4 M at one,
// against 15.9 M for 64.  The compiled QP shapes: qp_compiled().
static int plan_layout(const DevModel& M, KParams* k, bool task_only) {
  int off = 0;
  auto take = [&](int n) {
    int o = off;
    off += (n + 1) & ~1;  // keep 16-byte alignment
    return o;
  };
  const int nx = k->nx, ng = k->ng, np = k->np, m = k->m, nv = M.nv;
  if (task_only) {  // task_kernel: scalars + kinematics only
    k->oRed = take(64);
    k->oSc = take(32);
  } else {
  k->oP = take(np * np);
  k->oG = take(ng * nx);
  k->oQ = take(nx);
  k->oAB = take(nx);
  k->oL = take(m);
  k->oU = take(m);
  k->oD = take(nx);
  k->oE = take(m);
  k->oDi = take(nx);
  k->oEi = take(m);
  k->oRho = take(m);
  k->oX = take(nx);
  k->oZ = take(m);
  k->oY = take(m);
  k->oDY = take(m);
  k->oXT = take(nx);
  k->oZT = take(m);
  k->oT1 = take(m > nx ? m : nx);
  k->oT2 = take(m > nx ? m : nx);
  k->oRed = take(64);
  k->oSc = take(32);
  k->oBc = take(nx + ng > 32 ? nx + ng : 32);  // Ruiz factors (nx + ng), ADMM passes (ng + np), EQP (<= kEqpRegCap)
  }
  k->oHi = -1;
  if (!task_only && k->problem == 0 && M.kind == 1 && qp_compiled(nx, ng, np)) k->oHi = take(nx * nx);
  k->oU0 = off;
  if (!task_only && k->problem == 0) {
    // QPIK QP kernel: the union holds only what it uses -- the task record
    // view (q, J, xdd, grad m, grad d, the mobile Jacobian, the task
    // Jacobian), the factor (Schur blocks for the compiled shapes, K^-1
    // otherwise) and the polish (index lists, x / y candidates; the LDS
    // EQP only where a KKT can exceed the register EQP's kEqpRegCap).
    // FR3: ~10 KB per wave instead of ~20.
    int u = k->oU0;
    auto takeu = [&](int n) {
      int o = u;
      u += (n + 1) & ~1;
      return o;
    };
    k->kq = takeu(nv);
    k->kJ = takeu(6 * nv);
    k->kxdd = takeu(6);
    k->kmg = takeu(k->narm);
    k->kdg = takeu(nv);
    k->kSv = takeu(3 * kMaxWheels);
    k->kJt = takeu(6 * np);
    const int kin_end = u;
    const int fac_end = k->oU0 + (qp_compiled(nx, ng, np) ? np * np + ng * np + 4 * ng : nx * nx + nx * ng);
    // manipulator QPs: the register EQP's size; a larger reduced KKT fails
    // that polish attempt and ADMM continues (the oracle applies the same
    // cap).  Whole-body QPs have no variable bounds, so every variable is free
    // in the reduced KKT (N = nx + active rows): capped at 16 their polish
    // fails whenever 6 (XLS-FR3) / 8 (Husky-FR3) rows are active and the
    // instance runs to the tight ADMM fallback (up to ~3 000 iterations);
    // they get the LDS EQP for N > 16
    const int N = M.kind == 1 ? nx + ng : (nx + ng < kEqpRegCap ? nx + ng : kEqpRegCap);
    k->ncap = N;
    k->nbuf = (N + 7) & ~7;
    const int reg_pol = k->oU0 + 128 + m;  // Fidx/Ridx | xx | yy
    // (compiled whole-body shapes solve every polish KKT in range-space form,
    // eqp_range: its H^-1 g_a buffer instead of the LDS LDL^T's)
    const int lds_pol = k->oHi >= 0 ? k->oU0 + 256 + kEqpRegCap * nx
                        : (qp_compiled(nx, ng, np) && N <= kEqpRegCap) ? 0
                        : k->oU0 + 64 + 64 + 128 + k->nbuf * 5 + N * (N + 1) / 2;
    int end = kin_end;
    end = end > fac_end ? end : fac_end;
    end = end > reg_pol ? end : reg_pol;
    end = end > lds_pol ? end : lds_pol;
    k->lds_doubles = (end + 1) & ~1;  // 16-byte aligned: the second lane group's plan follows
    if (end * 8 > 160 * 1024) return set_err(DRC_ERR_UNSUPPORTED, "model too large for the per-wave LDS plan");
    return DRC_OK;
  }
  // kinematics view of the union
  int u = k->oU0;
  auto takeu = [&](int n) {
    int o = u;
    u += (n + 1) & ~1;
    return o;
  };
  k->kT = takeu((nv + 1) * 12);
  k->kZ = takeu((nv + 1) * 3);
  k->kTe = takeu(12);
  k->kJ = takeu(6 * nv);
  const int ng_ = M.ngeom > nv ? M.ngeom : nv;
  k->kTg = takeu(ng_ * 12);
  k->kq = takeu(nv);
  k->kqd = takeu(nv);
  k->kPd = takeu(M.npairs);
  k->kPf = takeu((M.npairs + 7) / 8);  // one byte per pair
  k->kxdd = takeu(6);
  k->kmg = takeu(k->narm);
  k->kdg = takeu(nv);
  k->kSv = takeu(3 * kMaxWheels);
  const bool epa = task_only && !k->cf;
  // QPID's task extras read Ai and W after the collision stage
  if (!epa || k->problem == 1) {
    k->kAi = takeu(36);
    k->kW = takeu(k->narm * 6);
  }
  if (k->problem == 1) {  // QPID stage data (task kernel) and dynamics (QP kernel)
    k->kJd = takeu(6 * nv);
    k->kDa = takeu(6 * k->narm);
    k->kVf = takeu(nv);
    k->kX6 = takeu(72 + 6 * k->narm + 2 * k->narm * k->narm);
    k->kGdv = takeu(k->narm + nv);
    k->kBias = takeu(8);
    k->kMq = takeu(k->na * k->na);
    k->kGq = takeu(k->na);
  }
  if (k->cf && k->cf != 3) {  // W, W2 (6 x nv), M^-1, nu, g, task vectors, then the serial COD work (+ its nv x 6 result)
    const int ws = 6 * nv + 36 + 6 * nv + 18 + 2 * nv + 6 * nv;
    k->kCf = takeu(2 * 6 * nv + nv * nv + 3 * nv + 48 + (ws > 160 ? ws : 160));
  }
  // Regions dead once the collision stage starts (manipulability work, the
  // QP kernel's task Jacobian), then the EPA polytope laid over them: they
  // share LDS, which keeps the QPIK task kernel within 20 KB per wave
  // (8 waves per CU).  The GJK candidate list lives in the polytope's space
  // too (it is consumed before EPA starts).
  const int scr0 = u;
  if (epa && k->problem != 1) {
    k->kAi = takeu(36);
    k->kW = takeu(k->narm * 6);
  }
  k->kA6 = takeu(36);
  k->kPart = takeu(k->narm * k->narm);
  k->kJt = takeu(6 * np);
  k->kScr = takeu(160);  // serial 6x6 COD work (pinv_cod_serial: 3n^2 + 3n)
  if (epa) {
    k->kEpa = scr0;
    const int ep = scr0 + ((static_cast<int>((sizeof(EpaPoly) + 7) / 8) + 1) & ~1);
    u = u > ep ? u : ep;
    // int list of the GJK candidates, in the polytope's face planes (fn, fd):
    // the candidate GJKs write the EPA seed stash (epa_stash: vertex slots
    // kEpaStashV0.., out[], nv) while later candidates are still being read,
    // so the list must not overlap those; the face planes are only written
    // once EPA starts, after the last candidate is consumed
    static_assert(offsetof(EpaPoly, fn) % 8 == 0 && offsetof(EpaPoly, fd) == offsetof(EpaPoly, fn) + sizeof(EpaPoly::fn),
                  "face planes: one contiguous double-aligned region");
    static_assert(sizeof(EpaPoly::fn) + sizeof(EpaPoly::fd) >= kMaxPairs * sizeof(int),
                  "the face planes hold a candidate list of kMaxPairs ints");
    static_assert(offsetof(EpaPoly, fn) >= sizeof(EpaPoly::vw) + sizeof(EpaPoly::va) &&
                      offsetof(EpaPoly, out) >= offsetof(EpaPoly, fd) + sizeof(EpaPoly::fd) &&
                      offsetof(EpaPoly, nv) > offsetof(EpaPoly, out),
                  "stash (vw / va slots, out[], nv) outside the candidate list");
    k->kCand = scr0 + static_cast<int>(offsetof(EpaPoly, fn) / 8);
    const int ce = k->kCand + (M.npairs + 1) / 2;
    u = u > ce ? u : ce;
  } else {
    k->kEpa = 0;
    k->kCand = takeu((M.npairs + 1) / 2);
  }
  int kin_end = u;
  // K^-1, and G K^-1 for the register ADMM (QPIK shapes); QPID runs the LDS path (K^-1 only)
  int kinv_end = k->oU0 + nx * nx + (k->problem == 1 ? 0 : nx * ng);
  // polish KKT: free variables + active G rows.  QPID's (<= 81) is capped at 48 —
  // typically 7 qdd + 7 tau + 7 equality rows + the few active CBF rows and free
  // slacks — which halves the per-wave LDS; a larger guess fails that polish try
  const int N = k->problem == 1 ? 48 : nx + ng;
  k->ncap = N;
  k->nbuf = N > 64 ? 128 : 64;
  int pol_end = k->oU0 + 64 + 64 + 128 + k->nbuf * 5 + N * (N + 1) / 2;
  int end = kin_end;
  if (!task_only) {
    end = end > kinv_end ? end : kinv_end;
    end = end > pol_end ? end : pol_end;
  }
  k->lds_doubles = end;
  if (end * 8 > 160 * 1024) return set_err(DRC_ERR_UNSUPPORTED, "model too large for the per-wave LDS plan");
  return DRC_OK;
}

static int make_kparams(const drc_model_impl* mm, const drc_qpik_params* p, int stages, KParams* k,
                        int problem = 0, int cf = 0) {
  const DevModel& M = mm->hm.dev;
  std::memset(k, 0, sizeof(*k));
  k->problem = problem;
  k->cf = cf;
  for (int i = 0; i < 6; ++i) {
    k->kp[i] = p->kp[i];
    k->kv[i] = p->kv[i];
  }
  k->ff = p->feedforward;
  k->alpha_cbf = p->alpha_cbf;
  k->w_reg = p->w_reg;
  k->slack_w = p->slack_w;
  k->man_min = p->man_min;
  k->dist_min = p->dist_min;
  k->t = p->t;
  k->t0 = p->t0;
  k->duration = p->duration;
  if (stages && p->frame_id == -1) {  // stage outputs without a task frame: last joint
    k->frame_joint = M.nv;
    static const double eye[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
    std::memcpy(k->frame_place, eye, sizeof(k->frame_place));
  } else {
    if (p->frame_id < 0 || p->frame_id >= M.nframes)
      return set_err(DRC_ERR_UNKNOWN_LINK, "params.frame_id does not name a link of the model");
    if (M.frame_joint[p->frame_id] == 0)
      return set_err(DRC_ERR_UNKNOWN_LINK, "task frame is attached to the universe (no joint moves it)");
    k->frame_joint = M.frame_joint[p->frame_id];
    std::memcpy(k->frame_place, M.frame_place[p->frame_id], sizeof(k->frame_place));
  }
  if (p->mode < DRC_MODE_QPIK || p->mode > DRC_MODE_QPIK_CUBIC) return set_err(DRC_ERR_INVALID_ARGUMENT, "bad mode");
  k->mode = p->mode;
  k->stages = stages;
  k->s = p->solver;
  k->nv = M.nv;
  if (M.kind == 0) {
    k->narm = M.nv;
    k->c0 = 0;
    k->np = M.nv;
    k->nx = 3 * M.nv + 2;  // QP_IK.cpp:24-28
    k->na = M.nv;
  } else {
    k->narm = M.n_arm;
    k->c0 = M.mani_start;
    k->np = M.n_arm + M.n_wheel;
    k->nx = k->np;  // MoMa QP_IK.cpp:20
    k->na = k->np;
  }
  k->ng = 2 * k->narm + 2;
  if (problem == 1) {  // QPID: QP_ID.cpp:11-63 / MoMa QP_ID.cpp:11-33
    k->nx = M.kind == 0 ? 6 * M.nv + 2 : 2 * k->na;
    k->ng = 4 * k->narm + 2 + k->na;
  }
  k->m = k->nx + k->ng;
  k->rJac = 0;
  k->rMan = 6 * M.nv;
  k->rDist = k->rMan + 1 + k->narm;
  k->rXdd = k->rDist + 1 + M.nv;
  k->rQ = k->rXdd + 6;
  k->rQd = k->rQ + M.nv;
  k->rBias = k->rQd + M.nv;
  k->rMgd = k->rBias + 6;
  k->rDgd = k->rMgd + 1;
  k->rLen = problem == 1 ? k->rDgd + 1 : k->rQd;
  k->xcd_map = 0;
  if (k->nx > 64 || k->ng > 64 || k->narm > 8 || k->m > 128)
    return set_err(DRC_ERR_UNSUPPORTED, "QP larger than one wavefront's row mapping");
  if (k->s.max_iter < 1 || k->s.check_termination < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "bad solver settings");
  return plan_layout(M, k, stages != 0);
}

static int launch(const drc_model_impl* cm, const drc_qpik_params* params, int stages, int64_t B, const double* q,
                  const double* qdot, const double* xt, const double* xdt, const double* xi, const double* xdi,
                  double* out, int32_t* status, int32_t* iters, double* pose, double* jac, double* man,
                  double* dist, int32_t* pair, double* xdd, void* stream, uint64_t* stamps = nullptr) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");  // 32-bit work-queue counters
  if (!q || !qdot || !xdt) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot and xdot_target are required");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required for QPIKStep/QPIKCubic");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required for QPIKCubic");
  if (!stages && (!out || !status)) return set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out and status are required");
  KParams kt, kq;
  int rc = make_kparams(m, params, 1, &kt);
  if (rc) return rc;
  if (!stages) {
    rc = make_kparams(m, params, 0, &kq);
    if (rc) return rc;
  }
  HIP_TRY(hipSetDevice(m->device));
  // product path: per-instance task records (rLen doubles padded to whole
  // 128-B lines) in a model-owned pool; the stage API writes [field][B]
  const int64_t stride = (kt.rLen + 15) & ~int64_t(15);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* rec = nullptr;
  int* hard = nullptr;           // lane-stage hard list, B ints
  uint8_t* hard_flag = nullptr;  // and its per-instance flags
  StreamCtx* cx = nullptr;
  DoneGuard done_guard{cx, st};
  // lane-per-instance task stage (lane_task.hpp) for the compiled joint counts
  const DevModel& dm = m->hm.dev;
  // (3, auto: stage-only calls, where nothing overlaps the task stage.  The
  // default is 0: a full QPIK call is faster with the wave-per-instance
  // kernel, which shares the CUs with the QP kernels of the other sub-batches
  // (DESIGN.md), and stage and QPIK calls then see the same GJK witnesses)
  const int ls = m->lane_stage;
  const bool lane = (ls == 1 || ls == 2 || (ls == 3 && stages)) && (dm.nv == 6 || dm.nv == 7) &&
                    dm.ncand_slots <= kMaxCandSlots;
  // fused up to 16 Ki instances: there a call is a few instances per wave, its
  // makespan the tail the fused kernel and the EPA-first order below shorten;
  // at full batch the overlapped sub-batch pipeline wins.  Measured at
  // B = 16 384 (fused / pipeline): FR3 +10.5 % (+33 % with the order), UR5e
  // +10 % with the order (-4.1 % without), XLS-FR3 +4.3 %, Husky-FR3 +5.9 %;
  // B = 32 768: FR3 +3.7 %, UR5e -13 %, XLS-FR3 -12 %; B = 65 536: FR3 -13 %,
  // UR5e -21 % (profiles/r06t_envab_fuse_*.jsonl, r06x_*, r06y_*).
  // DRC_FUSE_MAX overrides
  static const int64_t fuse_max = env_int("DRC_FUSE_MAX", 16384, 0);
  const bool fuse =
      m->fused && !stages && !lane && B <= fuse_max && kQpGroup == 64 && qp_compiled(kq.nx, kq.ng, kq.np);
  // penetration-prone instances first (order_kernel.hip) for calls whose
  // makespan is the EPA tail: manipulator calls of 2 049 .. 8 192 instances
  // (DRC_ORDER_MIN / _MAX), and every fused manipulator call above that (FR3
  // fused at B = 12 288 +38 %, 16 384 +20 %, profiles/r06v_envab_order*.jsonl).
  // Fewer: the 2 048-wave fused grid starts every instance at once anyway.
  // Pipeline calls above 8 192: the order gains less than it costs
  // (profiles/r06f_envab_order_*.jsonl).  Whole-body robots: their predictor
  // flags ~60 % of the instances, which orders nothing (XLS-FR3 B = 4 096
  // -2.6 %, profiles/r06j_envab_order_b4096.jsonl; FR3 +15.7 %, UR5e +7.7 %).
  // A caller's explicit order (drc_debug_instance_order) wins
  static const int64_t order_max = env_int("DRC_ORDER_MAX", 8192, 0);
  static const int64_t order_min = env_int("DRC_ORDER_MIN", 2049, 0);
  const bool dbg_order = m->d_order && m->order_n == B;
  const bool auto_order = !stages && !lane && !dbg_order && B >= order_min && (B <= order_max || fuse) &&
                          dm.kind == 0 && dm.ncand_slots > 0 && dm.ncand_slots <= kMaxCandSlots;
  int32_t* order_buf = nullptr;
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (!stages || lane) {
      const int64_t rec_bytes = stages ? 0 : stride * B * 8;
      const int64_t ord_off = (rec_bytes + B * 4 + B + 7) & ~int64_t(7);
      if (int r = ensure_pool(cx, ord_off + (auto_order ? B * 9 : 0))) return r;
      if (!stages) rec = reinterpret_cast<double*>(cx->pool);
      hard = reinterpret_cast<int*>(static_cast<char*>(cx->pool) + rec_bytes);
      hard_flag = reinterpret_cast<uint8_t*>(static_cast<char*>(cx->pool) + rec_bytes + B * 4);
      if (auto_order) order_buf = reinterpret_cast<int32_t*>(static_cast<char*>(cx->pool) + ord_off);
    }
  }
  // sub-batches of >= 4 Ki instances (a chunk of >= 16 Ki keeps the XCD-aware
  // order; smaller ones run grid-stride order): with one sub-batch the QP
  // kernel waits for the whole task kernel, with several they overlap
  // (Husky-FR3's 16 Ki batch)
  static const int64_t min_sub = env_int("DRC_MIN_SUBBATCH", 4096, 1);
  int S = 1;
  if (!stages && !fuse)
    for (int c = m->chunks; c > 1; --c)
      // four sub-batches only of >= 16 Ki instances each (Husky-FR3, B = 16 384:
      // 4 x 4 Ki 10.49 M against 3 x 5.5 Ki 11.14 M solves/s, r04z)
      if (B / c >= min_sub && (c < 4 || B / c >= 16384)) {
        S = c;
        break;
      }
  const bool timed = m->timing && !stages;
  std::vector<hipEvent_t> tev;
  // (timing events come from the model's pool: creating five to fourteen
  // events per call cost host time inside the bench's timed region)
  auto mkev = [&](hipEvent_t* e) -> int {
    {
      std::lock_guard<std::mutex> g(m->mu);
      if (!m->evpool.empty()) {
        *e = m->evpool.back();
        m->evpool.pop_back();
      } else {
        *e = nullptr;
      }
    }
    if (!*e) HIP_TRY(hipEventCreate(e));
    tev.push_back(*e);
    return DRC_OK;
  };
  {
    std::lock_guard<std::mutex> g(m->mu);
    while (static_cast<int>(m->ln.lanes.size()) < S) {
      hipStream_t ls;
      hipEvent_t je;
      HIP_TRY(hipStreamCreateWithFlags(&ls, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&je, hipEventDisableTiming));
      m->ln.lanes.push_back(ls);
      m->ln.joins.push_back(je);
    }
    while (lane && !stages && ls == 1 && static_cast<int>(m->ln.sides.size()) < S) {
      hipStream_t ss;
      hipEvent_t f, j;
      HIP_TRY(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&f, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&j, hipEventDisableTiming));
      m->ln.sides.push_back(ss);
      m->ln.side_fork.push_back(f);
      m->ln.side_join.push_back(j);
    }
    if (!m->ln.fork) HIP_TRY(hipEventCreateWithFlags(&m->ln.fork, hipEventDisableTiming));
  }
  // (one sub-batch: its own task-start / last events bracket the call, no
  // separate call events)
  hipEvent_t e_start = nullptr, e_end = nullptr, t0e = nullptr, t1e = nullptr, t2e = nullptr;
  if (timed && S > 1) {
    if (int r = mkev(&e_start)) return r;
    if (int r = mkev(&e_end)) return r;
    HIP_TRY(hipEventRecord(e_start, st));
  }
  done_guard.forks = &m->ln;  // (launch_mu held: the stream lists do not change under it)
  if (S > 1) HIP_TRY(hipEventRecord(m->ln.fork, st));
  for (int c = 0; c < S; ++c) {
    const int64_t b0 = B * c / S, b1 = B * (c + 1) / S, Bc = b1 - b0;
    // the last sub-batch runs on the caller's stream itself: S sub-batches take
    // S streams, so S = 4 still fits HIP's default 4 hardware queues per process
    const bool own = S > 1 && c < S - 1;
    hipStream_t cs = own ? m->ln.lanes[c] : st;
    if (own) HIP_TRY(hipStreamWaitEvent(cs, m->ln.fork, 0));
    KParams kt_c = kt, kq_c = kq;
    kt_c.xcd_map = kq_c.xcd_map = Bc >= 16384 ? 1 : 0;
    // persistent grids (work queues hand out the instances): 1 024 task and
    // 4 096 QP waves per sub-batch.  Re-swept on the r06 kernels (the QP
    // kernel's instances are now cheaper than the task kernel's): against
    // 2 048 / 2 048, FR3 +2.8 %, UR5e +2.0 %, XLS-FR3 +1.4 %
    // (profiles/r06ae_envab_grid.jsonl, r06af_envab_grid2.jsonl); DRC_GRID_TASK
    // / _QP override for such experiments
    // (clamped to >= 8 and a multiple of 8: with the XCD-aware order every
    // residue class blockIdx & 7 needs waves to drain its queue)
    static const int64_t cap_t = env_int("DRC_GRID_TASK", 1024, 8) & ~int64_t(7);
    static const int64_t cap_q = env_int("DRC_GRID_QP", 4096, 8) & ~int64_t(7);
    const int64_t gq = Bc < cap_q ? Bc : cap_q, gt = Bc < cap_t ? Bc : cap_t;
    IO io{Bc, b0, B, q, qdot, xt, xdt, xi, xdi, out, status, iters, pose, jac, man, dist, xdd, pair,
          rec ? rec + b0 * stride : nullptr, stride};
    io.stamps = stages ? nullptr : stamps;
    io.order = (!stages && !lane && dbg_order) ? m->d_order : nullptr;
    int* qc = cx->d_queue + c * StreamCtx::kSlotInts;  // c < 16 (drc_set_concurrency)
    // the whole slot (128 B, one aligned fill; 17 ints took two fill kernels)
    HIP_TRY(hipMemsetAsync(qc, 0, StreamCtx::kSlotInts * sizeof(int), cs));
    io.queue = qc;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    // kernel timing: every sub-batch's task and QP launches (each marker is a
    // queue packet between two kernels; a call of one sub-batch records two or
    // three: the five of r05 cost 6 % at FR3 B = 4 096.  Timing only the
    // caller-stream sub-batch of a four-sub-batch call saved 1.5 % but its
    // events then disagreed with rocprofv3's kernel averages by ~40 %, r05fin)
    const bool timed_c = timed;
    if (timed_c) {
      if (int r = mkev(&e0)) return r;
      if (int r = mkev(&e1)) return r;
      if (!fuse)  // the fused kernel has no QP launch of its own: its end is e1
        if (int r = mkev(&e2)) return r;
      HIP_TRY(hipEventRecord(e0, cs));
      t0e = e0;
      t1e = e1;
      t2e = fuse ? e1 : e2;
    }
    const size_t lds_t = static_cast<size_t>(kt_c.lds_doubles) * sizeof(double);
    const size_t lds_q = stages ? 0 : static_cast<size_t>(kq_c.lds_doubles) * sizeof(double);
    auto launch_task = [&](hipStream_t sm) -> int {
      HIP_TRY(static_cast<hipError_t>(launch_task_kernel(0, static_cast<unsigned>(gt), lds_t, sm, m->d_model, kt_c, io)));
      return DRC_OK;
    };
    auto launch_qp = [&]() -> int {
      io.queue = qc + 8;
      // compile-time QP shapes of the bundled robots; anything else runs the
      // runtime-sized instantiation (one LDS plan per lane group)
      HIP_TRY(static_cast<hipError_t>(launch_qp_kernel(static_cast<unsigned>(gq), lds_q, cs, m->d_model, kq_c, io)));
      return DRC_OK;
    };
    if (order_buf) {  // this sub-batch's order (hot count in the zeroed queue slot; hot list / flags after it)
      int32_t* hl = order_buf + B + b0;
      uint8_t* hf = reinterpret_cast<uint8_t*>(order_buf + 2 * B) + b0;
      HIP_TRY(static_cast<hipError_t>(launch_order_kernel(Bc, cs, m->d_model, io, qc + 24, hl, hf, order_buf)));
      io.order = order_buf;
    }
    if (fuse) {  // one fused task + QP kernel, the record in LDS
      static const int64_t cap_f = env_int("DRC_GRID_FUSED", 2048, 8) & ~int64_t(7);
      const int64_t gf = Bc < cap_f ? Bc : cap_f;
      const size_t lds_f =
          static_cast<size_t>(fused_lds_doubles(kt_c, kq_c)) *
          sizeof(double);
      io.queue = qc;
      HIP_TRY(static_cast<hipError_t>(
          launch_fused_kernel(static_cast<unsigned>(gf), lds_f, cs, m->d_model, kt_c, kq_c, io)));
      if (timed_c) HIP_TRY(hipEventRecord(e1, cs));
    } else if (!lane) {  // wave-per-instance task kernel on every instance, then the QP
      if (int r = launch_task(cs)) return r;
      if (timed_c) HIP_TRY(hipEventRecord(e1, cs));
      if (!stages)
        if (int r = launch_qp()) return r;
    } else {
      // lane stage for every instance; the wave-per-instance task kernel only
      // for the instances it hands back (hard list)
      io.hard_list = hard + b0;
      io.hard_n = qc + 16;
      io.hard_flag = stages ? nullptr : hard_flag + b0;
      const unsigned gl = static_cast<unsigned>((Bc + 63) / 64);  // one lane per instance
      HIP_TRY(static_cast<hipError_t>(launch_lane_task_kernel(dm.nv, gl, cs, m->d_model, kt_c, io)));
      if (timed_c) HIP_TRY(hipEventRecord(e1, cs));
      io.hard_mode = 1;
      if (stages || ls != 1) {  // hard task kernel, then one QP pass over every instance
        if (int r = launch_task(cs)) return r;
        io.hard_mode = 0;
        if (!stages)
          if (int r = launch_qp()) return r;
      } else {
        // hard task kernel on the side stream, overlapped with the QP of the
        // other instances; then the QP of the hard ones
        hipStream_t ss = m->ln.sides[c];
        HIP_TRY(hipEventRecord(m->ln.side_fork[c], cs));
        HIP_TRY(hipStreamWaitEvent(ss, m->ln.side_fork[c], 0));
        if (int r = launch_task(ss)) return r;
        HIP_TRY(hipEventRecord(m->ln.side_join[c], ss));
        io.hard_mode = 2;
        if (int r = launch_qp()) return r;
        HIP_TRY(hipStreamWaitEvent(cs, m->ln.side_join[c], 0));
        io.hard_mode = 1;
        if (int r = launch_qp()) return r;
      }
      io.hard_mode = 0;
    }
    if (timed_c && !fuse) HIP_TRY(hipEventRecord(e2, cs));
    if (own) HIP_TRY(hipEventRecord(m->ln.joins[c], cs));
  }
  for (int c = 0; c < S - 1; ++c) HIP_TRY(hipStreamWaitEvent(st, m->ln.joins[c], 0));
  if (timed) {
    if (S > 1) HIP_TRY(hipEventRecord(e_end, st));
    std::vector<hipEvent_t> ev = S > 1 ? tev : std::vector<hipEvent_t>{t0e, t2e, t0e, t1e, t2e};
    std::lock_guard<std::mutex> g(m->mu);
    m->events.push_back({ev, S});
  }
  done_guard.ok = true;
  return DRC_OK;
}

// QPID pipeline for one call: dynamics launch(es) -> task kernel (QPID stage
// data into the records) -> QPID kernel; or, with stages, the task kernel
// writing the stage outputs.  Model-owned scratch holds the records and the
// dynamics ([na*na][B] M, [na][B] g, MoMa also [nv][B] joint-order g).
static int launch_qpid(const drc_model_impl* cm, const drc_qpik_params* params, int stages, int64_t B,
                       const double* q, const double* qdot, const double* xt, const double* xdt, const double* xi,
                       const double* xdi, double* qdd, double* tau, int32_t* status, int32_t* iters, double* pose,
                       double* jac, double* man, double* dist, int32_t* pair, double* xdd, double* jdot,
                       double* qpid_st, double* gdv, void* stream) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (!q || !qdot || !xdt) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot and xdot_target are required");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required for QPIDStep/QPIDCubic");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required for QPIDCubic");
  if (!stages && (!qdd || !tau || !status)) return set_err(DRC_ERR_INVALID_ARGUMENT, "qddot_out, tau_out and status are required");
  KParams kt, kq;
  int rc = make_kparams(m, params, 1, &kt, 1);
  if (rc) return rc;
  if (!stages) {
    rc = make_kparams(m, params, 0, &kq, 1);
    if (rc) return rc;
  }
  const DevModel& d = m->hm.dev;
  HIP_TRY(hipSetDevice(m->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t stride = (kt.rLen + 15) & ~int64_t(15);
  const int na = kt.na, nv = d.nv;
  const int64_t dyn_words = stages ? 0 : (int64_t(na) * na + na + (d.kind == 1 ? nv : 0)) * B;
  double *rec = nullptr, *dM = nullptr, *dG = nullptr, *dGf = nullptr;
  StreamCtx* cx = nullptr;
  DoneGuard done_guard{cx, st};
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (!stages)
      if (int r = ensure_pool(cx, (stride * B + dyn_words) * 8)) return r;
  }
  if (!stages) {
    rec = reinterpret_cast<double*>(cx->pool);
    dM = rec + stride * B;
    dG = dM + int64_t(na) * na * B;
    dGf = d.kind == 1 ? dG + int64_t(na) * B : nullptr;
    // getMassMatrix / getGravity (or the *Actuated getters) the equality rows use
    rc = launch_dynamics(m->d_model, d, d.kind == 1, B, q, qdot, dM, nullptr, dG, nullptr, nullptr, nullptr, st);
    if (!rc && d.kind == 1) rc = launch_dynamics(m->d_model, d, false, B, q, qdot, nullptr, nullptr, dGf, nullptr, nullptr, nullptr, st);
    if (rc) return set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  }
  const int64_t grid = B < 8192 ? B : 8192;
  KParams kt_c = kt, kq_c = kq;
  kt_c.xcd_map = kq_c.xcd_map = B >= 16384 ? 1 : 0;
  IO io{B, 0, B, q, qdot, xt, xdt, xi, xdi, qdd, status, iters, pose, jac, man, dist, xdd, pair, rec, stride};
  io.dM = dM;
  io.dG = dG;
  io.dGf = dGf;
  io.out2 = tau;
  io.st_jdot = jdot;
  io.st_qpid = qpid_st;
  io.st_gdv = gdv;
  int* qc = cx->d_queue + StreamCtx::kQueueSlotQpid * StreamCtx::kSlotInts;
  HIP_TRY(hipMemsetAsync(qc, 0, 16 * sizeof(int), st));
  io.queue = qc;
  HIP_TRY(static_cast<hipError_t>(launch_task_kernel(1, static_cast<unsigned>(grid),
                                                     static_cast<size_t>(kt_c.lds_doubles) * sizeof(double), st,
                                                     m->d_model, kt_c, io)));
  if (!stages) {
    io.queue = qc + 8;
    const size_t lds = static_cast<size_t>(kq_c.lds_doubles) * sizeof(double);
    HIP_TRY(static_cast<hipError_t>(launch_qpid_kernel(static_cast<unsigned>(grid), lds, st, m->d_model, kq_c, io)));
  }
  done_guard.ok = true;
  return DRC_OK;
}

// Closed-form controllers: [dynamics (OSF: M^-1, g)] -> task_kernel<2>.
static int launch_closed_form(const drc_model_impl* cm, const drc_qpik_params* params, int cf, int64_t B,
                              const double* q, const double* qdot, const double* xt, const double* xdt,
                              const double* xi, const double* xdi, const double* nullv, double* out, void* stream,
                              double* pose = nullptr, double* jac = nullptr, double* xdot = nullptr) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (cf == 3) {  // kinematics only (drc_kinematics_batch): any model kind, no task targets
    if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
    if (B == 0) return DRC_OK;
    if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
    if (!q || (xdot && !qdot)) return set_err(DRC_ERR_INVALID_ARGUMENT, "q (and qdot for xdot) required");
    KParams kt;
    drc_qpik_params pp = *params;
    pp.mode = DRC_MODE_QPIK;
    int rc = make_kparams(m, &pp, 1, &kt, 2, 3);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    StreamCtx* cx = nullptr;
    DoneGuard done_guard{cx, st};
    {
      std::lock_guard<std::mutex> g(m->mu);
      if (int r = stream_ctx(m, st, &cx)) return r;
    }
    const int64_t grid = B < 8192 ? B : 8192;
    kt.xcd_map = B >= 16384 ? 1 : 0;
    // qdot may be NULL when xdot is not requested.  The stage still loads a
    // qdot vector (its J qdot product is then discarded, never stored), so q
    // stands in as a readable buffer of the same shape; with xdot requested
    // the caller's qdot is required (checked above)
    IO io{B, 0, B, q, qdot ? qdot : q, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, pose, jac,
          nullptr, nullptr, xdot, nullptr, nullptr, 0};
    // fixed assignment when every wave has one instance: no counter reset to enqueue
    io.queue = B > grid ? cx->d_queue + StreamCtx::kQueueSlotCf * StreamCtx::kSlotInts : nullptr;
    if (io.queue) HIP_TRY(hipMemsetAsync(io.queue, 0, 8 * sizeof(int), st));
    HIP_TRY(static_cast<hipError_t>(launch_task_kernel(2, static_cast<unsigned>(grid),
                                                       static_cast<size_t>(kt.lds_doubles) * sizeof(double), st,
                                                       m->d_model, kt, io)));
    done_guard.ok = true;
    return DRC_OK;
  }
  if (m->hm.dev.kind != 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "CLIK / OSF are Manipulator::RobotController entries");
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (!q || !qdot || !xdt || !out) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot, xdot_target and out are required");
  if (cf == 1 && params->mode == DRC_MODE_QPIK) return set_err(DRC_ERR_INVALID_ARGUMENT, "CLIK has Step and Cubic forms only");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi)) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required");
  drc_qpik_params pp = *params;
  for (int i = 0; i < 6; ++i) pp.kv[i] = cf == 1 ? 0.0 : params->kv[i];  // CLIK: Kp e + xdot_target (:168)
  pp.feedforward = cf == 1 ? 1.0 : 0.0;                                 // OSF: Kp e + Kv edot (:243)
  KParams kt;
  int rc = make_kparams(m, &pp, 1, &kt, 2, cf);
  if (rc) return rc;
  const DevModel& d = m->hm.dev;
  HIP_TRY(hipSetDevice(m->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double *dMi = nullptr, *dG = nullptr;
  StreamCtx* cx = nullptr;
  DoneGuard done_guard{cx, st};
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (cf == 2) {
      if (int r = ensure_pool(cx, (int64_t(d.nv) * d.nv + d.nv) * B * 8)) return r;
      if (cx->dyn_list_cap < B + 1) {
        if (cx->dyn_list) HIP_TRY(hipFree(cx->dyn_list));
        cx->dyn_list = nullptr;
        cx->dyn_list_cap = 0;
        HIP_TRY(hipMalloc(&cx->dyn_list, (B + 1) * sizeof(int)));
        cx->dyn_list_cap = B + 1;
      }
    }
  }
  if (cf == 2) {  // getMassMatrixInv (PinvCOD(M)) and getGravity (robot_data.cpp:111-118)
    dMi = reinterpret_cast<double*>(cx->pool);
    dG = dMi + int64_t(d.nv) * d.nv * B;
    rc = launch_dynamics(m->d_model, d, false, B, q, qdot, nullptr, dMi, dG, nullptr, nullptr, cx->dyn_list, st);
    if (rc) return set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  }
  const int64_t grid = B < 8192 ? B : 8192;
  kt.xcd_map = B >= 16384 ? 1 : 0;
  IO io{B, 0, B, q, qdot, xt, xdt, xi, xdi, out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, 0};
  io.dM = dMi;
  io.dG = dG;
  io.cf_null = nullv;
  io.queue = cx->d_queue + StreamCtx::kQueueSlotCf * StreamCtx::kSlotInts;
  HIP_TRY(hipMemsetAsync(io.queue, 0, 8 * sizeof(int), st));
  HIP_TRY(static_cast<hipError_t>(launch_task_kernel(2, static_cast<unsigned>(grid),
                                                     static_cast<size_t>(kt.lds_doubles) * sizeof(double), st,
                                                     m->d_model, kt, io)));
  done_guard.ok = true;
  return DRC_OK;
}

}  // namespace drc_amd

using drc_amd::drc_model_impl;
struct drc_model : drc_model_impl {};

extern "C" {

const char* drc_error_string(int code) {
  switch (code) {
    case DRC_OK: return "ok";
    case DRC_ERR_INVALID_ARGUMENT: return "invalid argument";
    case DRC_ERR_FILE: return "file does not exist";
    case DRC_ERR_PARSE: return "parse error";
    case DRC_ERR_UNSUPPORTED: return "unsupported model";
    case DRC_ERR_UNKNOWN_LINK: return "link name not found in URDF";
    case DRC_ERR_HIP: return "HIP runtime error";
    case DRC_ERR_SIZE_MISMATCH: return "size mismatch";
    default: return "unknown error";
  }
}
const char* drc_last_error(void) { return drc_amd::g_last_error.c_str(); }

#ifndef DRC_BUILD_ID
#define DRC_BUILD_ID "unknown"
#endif
const char* drc_build_id(void) { return DRC_BUILD_ID; }

int drc_debug_lds_plan(drc_model* m, const drc_qpik_params* params, int problem, int* task_bytes, int* qp_bytes,
                       int* fused_bytes) {
  if (!m || !params || !task_bytes || !qp_bytes || !fused_bytes) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  if (problem != 0 && problem != 1) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "problem must be 0 (QPIK) or 1 (QPID)");
  drc_amd::KParams kt, kq;
  if (int rc = drc_amd::make_kparams(m, params, 1, &kt, problem)) return rc;
  if (int rc = drc_amd::make_kparams(m, params, 0, &kq, problem)) return rc;
  *task_bytes = kt.lds_doubles * 8;
  *qp_bytes = kq.lds_doubles * 8;
  // the fused kernel (QPIK only): the larger plan plus the task record
  *fused_bytes = problem == 0 ? drc_amd::fused_lds_doubles(kt, kq) * 8 : 0;
  return DRC_OK;
}

int drc_debug_waves(drc_model* m, const drc_qpik_params* params, int* task_waves, int* qp_waves) {
  if (!m || !params || !task_waves || !qp_waves) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  drc_amd::KParams kt;
  if (int rc = drc_amd::make_kparams(m, params, 1, &kt, 0)) return rc;
  *task_waves = drc_amd::task_waves_per_simd(0, static_cast<size_t>(kt.lds_doubles) * 8);
  *qp_waves = drc_amd::qp_waves_per_simd();
  return DRC_OK;
}

int drc_debug_host_timeline(drc_model* m, int enable, int64_t* out, int64_t cap, int64_t* n) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> g(m->host_mu);
  const int64_t rows = static_cast<int64_t>(m->tl.size() / 5);
  if (n) *n = rows;
  if (out)
    for (int64_t i = 0; i < rows * 5 && i < cap * 5; ++i) out[i] = m->tl[static_cast<size_t>(i)];
  m->tl.clear();
  m->tl_on = enable != 0;
  return DRC_OK;
}

int drc_debug_kernel_timing(drc_model* m, int enable) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  m->timing = enable != 0;
  return DRC_OK;
}

int drc_debug_kernel_times(drc_model* m, double* wall_ms, double* task_ms, double* qp_ms, int* calls) {
  if (!m || !wall_ms || !task_ms || !qp_ms || !calls) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> g(m->mu);
  double tw = 0, t0 = 0, t1 = 0;
  for (auto& evs : m->events) {  // {start, end, task start, task end, qp end}, sub-batches
    const std::vector<hipEvent_t>& ev = evs.first;
    float a = 0;
    if (hipEventSynchronize(ev[1]) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventSynchronize");
    if (hipEventElapsedTime(&a, ev[0], ev[1]) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventElapsedTime");
    tw += a;
    for (size_t c = 2; c + 2 < ev.size(); c += 3) {
      float x = 0, y = 0;
      if (hipEventElapsedTime(&x, ev[c], ev[c + 1]) != hipSuccess ||
          hipEventElapsedTime(&y, ev[c + 1], ev[c + 2]) != hipSuccess)
        return drc_amd::set_err(DRC_ERR_HIP, "hipEventElapsedTime");
      t0 += x;
      t1 += y;
    }
  }
  *calls = static_cast<int>(m->events.size());
  for (auto& evs : m->events) {  // completed: reusable (each event once: a call's list may name one twice)
    std::vector<hipEvent_t> u = evs.first;
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    for (hipEvent_t e : u) m->evpool.push_back(e);
  }
  m->events.clear();
  *wall_ms = tw;
  *task_ms = t0;
  *qp_ms = t1;
  return DRC_OK;
}

int drc_set_fusion(drc_model* m, int enable) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> g(m->launch_mu);
  m->fused = enable != 0;
  return DRC_OK;
}

int drc_set_concurrency(drc_model* m, int chunks) {
  if (!m || chunks < 1 || chunks > 16) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "chunks must be 1..16");
  std::lock_guard<std::mutex> g(m->mu);
  m->chunks = chunks;
  return DRC_OK;
}

int drc_debug_lane_stage(drc_model* m, int enable) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> g(m->launch_mu);
  m->lane_stage = enable < 0 ? 0 : (enable > 3 ? 3 : enable);
  return DRC_OK;
}

int drc_debug_instance_order(drc_model* m, const int32_t* order, int64_t n) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> g(m->launch_mu);
  HIP_TRY(hipSetDevice(m->device));
  if (m->d_order) {
    HIP_TRY(hipDeviceSynchronize());  // calls in flight may still read it
    HIP_TRY(hipFree(m->d_order));
  }
  m->d_order = nullptr;
  m->order_n = 0;
  if (!order || n <= 0) return DRC_OK;
  std::vector<char> seen(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (order[i] < 0 || order[i] >= n || seen[order[i]]) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "not a permutation");
    seen[order[i]] = 1;
  }
  HIP_TRY(hipMalloc(&m->d_order, n * sizeof(int32_t)));
  HIP_TRY(hipMemcpy(m->d_order, order, n * sizeof(int32_t), hipMemcpyHostToDevice));
  m->order_n = n;
  return DRC_OK;
}

#ifdef DRC_PHASE_TIMING
// diagnostic build only: accumulated per-phase s_memtime cycles (32 slots)
int drc_debug_phase_cycles(unsigned long long* out, int reset) {
  for (int i = 0; i < 64; ++i) out[i] = 0;
  if (drc_amd::phase_cycles_task(out, reset) || drc_amd::phase_cycles_qp(out, reset) ||
      drc_amd::phase_cycles_qpid(out, reset) || drc_amd::phase_cycles_fused(out, reset))
    return DRC_ERR_HIP;
  return DRC_OK;
}
#endif

int drc_model_create_manipulator(const char* urdf, const char* srdf, const char* packages, int device,
                                 drc_model** out) {
  (void)packages;  // collision meshes are not supported: primitives only
  if (!urdf || !out) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  auto* m = new drc_model();
  std::string err;
  int rc = drc_amd::build_model_from_urdf(urdf, srdf ? srdf : "", &m->hm, &err);
  if (rc) {
    delete m;
    return drc_amd::set_err(rc, err);
  }
  m->hm.dev.kind = 0;
  m->device = device;
  rc = drc_amd::upload(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return DRC_OK;
}

int drc_model_create_mobile_manipulator(const drc_kinematic_param* param, const drc_joint_index* ji,
                                        const drc_actuator_index* ai, const char* urdf, const char* srdf,
                                        const char* packages, int device, drc_model** out) {
  (void)packages;
  if (!param || !ji || !ai || !urdf || !out) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  auto* m = new drc_model();
  std::string err;
  int rc = drc_amd::build_model_from_urdf(urdf, srdf ? srdf : "", &m->hm, &err);
  if (rc) {
    delete m;
    return drc_amd::set_err(rc, err);
  }
  drc_amd::DevModel& d = m->hm.dev;
  int W = 0;
  rc = drc_amd::mobile_fk_jacobian(*param, &W, d.J_mobile);
  if (rc) {
    delete m;
    return rc;
  }
  d.drive = param->type;
  d.wheel_radius = param->wheel_radius;
  d.wheel_offset = param->wheel_offset;
  for (int i = 0; i < drc_amd::kMaxWheels / 2; ++i)
    for (int k = 0; k < 2; ++k) d.caster_pos[i][k] = param->base2wheel_positions[i][k];
  if (param->type == DRC_DRIVE_CASTER && !(param->wheel_offset != 0)) {
    delete m;
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive needs a nonzero wheel_offset");
  }
  // MobileManipulator::RobotData ctor (mobile_manipulator/robot_data.cpp:18-25)
  const int virtual_dof = 3;
  d.kind = 1;
  d.n_wheel = W;
  d.n_arm = d.nv - (virtual_dof + W);  // every joint 1-DoF, no extra joints
  d.virtual_start = ji->virtual_start;
  d.mani_start = ji->mani_start;
  d.mobi_start = ji->mobi_start;
  d.act_mani_start = ai->mani_start;
  d.act_mobi_start = ai->mobi_start;
  d.dyn_origin = ji->virtual_start + 3;  // the base (yaw joint) origin: keeps spatial moments small
  if (d.n_arm < 1 || d.n_arm > 8 || ji->virtual_start + 3 > d.nv || ji->mani_start + d.n_arm > d.nv ||
      ji->mobi_start + W > d.nv || ai->mani_start + d.n_arm > d.n_arm + W || ai->mobi_start + W > d.n_arm + W) {
    delete m;
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "JointIndex/ActuatorIndex inconsistent with the URDF dof");
  }
  m->kparam = *param;
  m->jidx = *ji;
  m->aidx = *ai;
  m->device = device;
  rc = drc_amd::upload(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return DRC_OK;
}

int drc_model_release_stream(drc_model* m, void* stream) {
  using drc_amd::set_err;
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  std::lock_guard<std::mutex> g(m->mu);
  HIP_TRY(hipSetDevice(m->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (size_t i = 0; i < m->ctxs.size(); ++i)
    if (m->ctxs[i]->stream == st) {
      HIP_TRY(hipStreamSynchronize(st));  // the stream is still valid: its work on the context drains first
      drc_amd::free_ctx(m->ctxs[i].get());
      m->ctxs.erase(m->ctxs.begin() + static_cast<std::ptrdiff_t>(i));
      break;
    }
  return DRC_OK;
}

void drc_model_destroy(drc_model* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  (void)hipDeviceSynchronize();
  for (auto& c : m->ctxs) drc_amd::free_ctx(c.get());
  drc_amd::free_lanes(&m->ln);
  if (m->d_model) (void)hipFree(m->d_model);
  if (m->d_order) (void)hipFree(m->d_order);
  if (m->hstream) (void)hipStreamSynchronize(m->hstream), (void)hipStreamDestroy(m->hstream);
  if (m->stage) (void)hipFree(m->stage);
  if (m->pinned) (void)hipHostFree(m->pinned);
  if (m->hdone) (void)hipEventDestroy(m->hdone);
  for (auto& evs : m->events) {
    std::vector<hipEvent_t> u = evs.first;
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    for (hipEvent_t e : u) (void)hipEventDestroy(e);
  }
  for (hipEvent_t e : m->evpool) (void)hipEventDestroy(e);
  delete m;
}

int drc_model_info(const drc_model* m, int* dof, int* act, int* mani, int* mobi, int* ngeom, int* npairs) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const drc_amd::DevModel& d = m->hm.dev;
  if (dof) *dof = d.nv;
  if (act) *act = d.kind == 1 ? d.n_arm + d.n_wheel : d.nv;
  if (mani) *mani = d.kind == 1 ? d.n_arm : d.nv;
  if (mobi) *mobi = d.kind == 1 ? d.n_wheel : 0;
  if (ngeom) *ngeom = d.ngeom;
  if (npairs) *npairs = d.npairs;
  return DRC_OK;
}

int drc_model_limits(const drc_model* m, double* q_lb, double* q_ub, double* qd_lb, double* qd_ub) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const drc_amd::DevModel& d = m->hm.dev;
  for (int i = 0; i < d.nv; ++i) {
    if (q_lb) q_lb[i] = d.lower[i];
    if (q_ub) q_ub[i] = d.upper[i];
    if (qd_lb) qd_lb[i] = -d.vel[i];
    if (qd_ub) qd_ub[i] = d.vel[i];
  }
  return DRC_OK;
}

int drc_model_find_frame(const drc_model* m, const char* name, int* id) {
  if (!m || !name || !id) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  const auto& names = m->hm.frame_names;
  for (size_t i = 0; i < names.size(); ++i)
    if (names[i] == name) {
      *id = static_cast<int>(i);
      return DRC_OK;
    }
  *id = -1;
  return drc_amd::set_err(DRC_ERR_UNKNOWN_LINK, std::string("Link name ") + name + " not found in URDF.");
}

int drc_model_mobile_fk_jacobian(const drc_model* m, double* J) {
  if (!m || !J) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  const drc_amd::DevModel& d = m->hm.dev;
  if (d.kind != 1) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "not a mobile manipulator");
  if (d.drive == drc_amd::kDriveCaster)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT,
                            "caster drive: J_mobile depends on the steer angles (drc_mobile_fk_jacobian)");
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < d.n_wheel; ++c) J[r * d.n_wheel + c] = d.J_mobile[r][c];
  return DRC_OK;
}

int drc_mobile_fk_jacobian(const drc_kinematic_param* p, const double* wheel_pos, double* J, int* n_wheels) {
  if (!p || !J || !n_wheels) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  if (p->type == DRC_DRIVE_CASTER && !wheel_pos)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive: wheel positions required");
  double Jm[3][drc_amd::kMaxWheels];
  int W = 0;
  if (int rc = drc_amd::mobile_fk_jacobian(*p, &W, Jm, wheel_pos)) return rc;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < W; ++c) J[r * W + c] = Jm[r][c];
  *n_wheels = W;
  return DRC_OK;
}

int drc_mobile_ik_jacobian(const drc_kinematic_param* p, const double* wheel_pos, double* J, int* n_wheels) {
  if (!p || !J || !n_wheels) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  if (p->type == DRC_DRIVE_CASTER && !wheel_pos)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive: wheel positions required");
  return drc_amd::mobile_ik_jacobian(*p, wheel_pos, J, n_wheels);
}

int drc_default_qpik_params(const drc_model* m, int exact, drc_qpik_params* p) {
  if (!m || !p) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  std::memset(p, 0, sizeof(*p));
  const bool moma = m->hm.dev.kind == 1;
  for (int i = 0; i < 6; ++i) {
    p->kp[i] = moma ? 400 : 100;  // robot_controller.cpp:12 ; MoMa :15
    p->kv[i] = moma ? 0 : 20;     // MoMa QPIKStep: Kp*e + xdot_target (:177)
  }
  p->feedforward = moma ? 1.0 : 0.0;
  p->alpha_cbf = 50;
  p->w_reg = moma ? 0.01 : 1.0;
  p->slack_w = 1000;
  p->man_min = 0.01;
  p->dist_min = 0.05;
  p->mode = DRC_MODE_QPIK_STEP;
  p->frame_id = -1;
  drc_solver_settings& s = p->solver;
  s.rho = 0.1;
  s.sigma = 1e-6;
  s.alpha = 1.6;
  s.eps_abs = 1e-3;
  s.eps_rel = 1e-3;
  s.eps_prim_inf = 1e-4;
  s.max_iter = 4000;
  s.check_termination = 25;
  s.scaling = 10;
  s.adaptive_rho = 1;
  s.adaptive_rho_interval = 25;
  s.adaptive_rho_tolerance = 5;
  s.polish = exact ? 1 : 0;
  s.polish_refine_iter = 3;
  s.delta = 1e-6;
  s.exact = exact ? 1 : 0;
  s.eps_exact = 1e-9;
  s.eps_fallback = 1e-7;
  // exact mode: the ADMM iterate only seeds the certified polish's first
  // active-set guess, so how often it is tried is a speed choice.  With the
  // projected-Jacobi guess the first polish paid off at iteration 20 (+1-2.5 %
  // against 25, profiles/r05h_envab_check20.jsonl); with the infeasible-phase
  // drop rule it pays off far earlier: manipulators at 8 (FR3 +7 %, UR5e +4 %;
  // below 8 UR5e loses), the whole-body QPs at 2 (XLS-FR3 +12 %, Husky-FR3
  // +6 %; profiles/r05ae-ag_envab_check*.jsonl).  The oracle's exact mode uses
  // the same intervals.  DRC_EXACT_CHECK overrides both (A/B experiments)
  static const int64_t exact_check_env = drc_amd::env_int("DRC_EXACT_CHECK", 0, 0);
  const int64_t exact_check = exact_check_env > 0 ? exact_check_env : (moma ? 2 : 8);
  // OSQP's 3 refinement steps.  2 certify the same attempts at eps_exact
  // (tools/polish_census.py --refine; 1 fails half) and measured UR5e +1.1 %,
  // FR3 +0.1 % (profiles/r05b_envab.jsonl), but leave ~2e-9 in q-dot on some
  // instances (a golden fixture moved by 2.5e-9): not taken for that
  static const int64_t exact_refine = drc_amd::env_int("DRC_EXACT_REFINE", 3, 0);
  // Ruiz passes in exact mode: 1 (manipulators) / 2 (whole-body) instead of
  // OSQP's 10.  The ADMM only seeds the certified polish there (8 / 2
  // iterations), and the certified point is the QP's unique optimum whatever
  // the scaling; a pass or two equilibrate enough for the polish to certify at
  // its first attempt, the rest cost (whole-body QPs run all 10: a balanced
  // row's factor converges geometrically and never reaches exactly 1).
  // Measured, one box, 2 against 10: FR3 +2.6 %, UR5e +2.1 %, Husky-FR3
  // +2.9 %, XLS-FR3 +9.9 %, Caster-FR3 +10.5 %; one pass leaves the whole-body
  // polish failing (3.6 M solves/s), none fails everywhere
  // (profiles/r06f_envab_exact_scaling.jsonl, r06g_envab_exact_scaling.jsonl);
  // 1 against 2 on the manipulators: FR3 +0.6 %, UR5e +1.8 %, FR3 B = 4 096
  // +1.2 % (profiles/r06al_envab_scal1*.jsonl).  The oracle's exact mode uses
  // the same counts.  DRC_EXACT_SCALING overrides both kinds (A/B experiments)
  static const int64_t exact_scaling_env = drc_amd::env_int("DRC_EXACT_SCALING", 0, 0);
  const int64_t exact_scaling = exact_scaling_env > 0 ? exact_scaling_env : (moma ? 2 : 1);
  if (exact) {
    s.check_termination = static_cast<int>(exact_check);
    s.polish_refine_iter = static_cast<int>(exact_refine);
    s.scaling = static_cast<int>(exact_scaling);
  }
  return DRC_OK;
}

int drc_qpik_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                   int32_t* status, int32_t* iters, void* stream) {
  return drc_amd::launch(m, p, 0, B, q, qdot, xt, xdt, xi, xdi, out, status, iters, nullptr, nullptr, nullptr,
                         nullptr, nullptr, nullptr, stream);
}

int drc_qpik_stages_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q,
                          const double* qdot, const double* xt, const double* xdt, const double* xi,
                          const double* xdi, double* pose, double* jac, double* man, double* dist, int32_t* pair,
                          double* xdd, void* stream) {
  return drc_amd::launch(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, nullptr, nullptr, nullptr, pose, jac, man, dist,
                         pair, xdd, stream);
}


// ---- QPID -------------------------------------------------
int drc_default_qpid_params(const drc_model* m, int exact, drc_qpik_params* p) {
  int rc = drc_default_qpik_params(m, exact, p);
  if (rc) return rc;
  const bool moma = m->hm.dev.kind == 1;
  for (int i = 0; i < 6; ++i) {
    p->kp[i] = moma ? 400 : 100;  // robot_controller.cpp:12-13; MoMa :15-16
    p->kv[i] = moma ? 40 : 20;    // QPIDStep: Kp e + Kv (xdot_target - xdot) (:347; MoMa :230)
  }
  p->feedforward = 0;
  p->w_reg = 0;  // QP_ID.cpp:102: the regulariser is commented out
  // P is singular on null(J); OSQP's polish delta 1e-6 cannot certify at
  // eps_exact there, so parity mode regularises the polish with 1e-10
  if (exact) p->solver.delta = 1e-10;
  p->solver.check_termination = 25;  // QPID keeps OSQP's check interval,
  p->solver.polish_refine_iter = 3;   // refinement count and Ruiz passes in every mode
  p->solver.scaling = 10;             // (its optimum is a face: the scaling picks the point on it)
  return DRC_OK;
}

int drc_qpid_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, double* qddot_out,
                   double* tau_out, int32_t* status, int32_t* iters, void* stream) {
  return drc_amd::launch_qpid(m, p, 0, B, q, qdot, xt, xdt, xi, xdi, qddot_out, tau_out, status, iters, nullptr,
                              nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int drc_qpid_stages_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q,
                          const double* qdot, const double* xt, const double* xdt, const double* xi,
                          const double* xdi, double* pose, double* jac, double* man, double* dist, int32_t* pair,
                          double* xddot_des, double* jdot, double* qpid_terms, double* graddot, void* stream) {
  return drc_amd::launch_qpid(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, nullptr, nullptr, nullptr, nullptr, pose, jac,
                              man, dist, pair, xddot_des, jdot, qpid_terms, graddot, stream);
}

int drc_qpid_stages_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                         const double* xt, const double* xdt, const double* xi, const double* xdi, double* pose,
                         double* jac, double* man, double* dist, int32_t* pair, double* xddot_des, double* jdot,
                         double* qpid_terms, double* graddot) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, na = d.kind == 1 ? d.n_arm : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[6] = {q, qdot, xt, xdt, xi, xdi};
  const int64_t rin[6] = {n, n, 12, 6, 12, 6};
  double* outs[8] = {pose, jac, man, dist, xddot_des, jdot, qpid_terms, graddot};
  const int64_t rout[8] = {12, 6 * n, 1 + na, 1 + n, 6, 6 * n, 8, na + n};
  int64_t words = (B + 1) / 2;
  for (int i = 0; i < 6; ++i) words += src[i] ? rin[i] * B : 0;
  for (int i = 0; i < 8; ++i) words += outs[i] ? rout[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 6; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rin[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rin[i] * B;
    }
  double* dout[8] = {nullptr};
  for (int i = 0; i < 8; ++i)
    if (outs[i]) {
      dout[i] = dp;
      dp += rout[i] * B;
    }
  int32_t* dpair = pair ? reinterpret_cast<int32_t*>(dp) : nullptr;
  int rc = drc_qpid_stages_batch(m, p, B, din[0], din[1], din[2], din[3], din[4], din[5], dout[0], dout[1], dout[2],
                                 dout[3], dpair, dout[4], dout[5], dout[6], dout[7], m->hstream);
  if (rc) return rc;
  for (int i = 0; i < 8; ++i)
    if (outs[i]) HIP_TRY(hipMemcpyAsync(outs[i], dout[i], rout[i] * B * 8, hipMemcpyDeviceToHost, m->hstream));
  if (pair) HIP_TRY(hipMemcpyAsync(pair, dpair, B * 4, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

}  // extern "C"

// ---- host-buffer entry points (synchronous; staged through device memory) --
namespace drc_amd {
struct HostIO {
  const double* src[6];  // q, qdot, xt, xdt, xi, xdi
  int64_t rows[6];
};

// Device staging buffer and its pinned host mirror, both >= `words` doubles
// (the caller holds m->host_mu).
static int ensure_staging(drc_model* m, int64_t words) {
  const int64_t bytes = words * 8;
  if (m->stage_bytes < bytes) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    if (hipMalloc(&m->stage, bytes) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipMalloc (staging)");
    m->stage_bytes = bytes;
  }
  if (m->pinned_bytes < bytes) {
    if (m->pinned) (void)hipHostFree(m->pinned);
    m->pinned = nullptr;
    m->pinned_bytes = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&m->pinned), bytes, hipHostMallocDefault) != hipSuccess)
      return drc_amd::set_err(DRC_ERR_HIP, "hipHostMalloc (staging)");
    m->pinned_bytes = bytes;
  }
  if (!m->hdone && hipEventCreateWithFlags(&m->hdone, hipEventDisableTiming) != hipSuccess)
    return drc_amd::set_err(DRC_ERR_HIP, "hipEventCreate (host entries)");
  if (!m->hstream && hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking) != hipSuccess)
    return drc_amd::set_err(DRC_ERR_HIP, "hipStreamCreate");
  return DRC_OK;
}

// A synchronous host-buffer call in one round trip: the inputs are packed
// into the pinned mirror and sent in one transfer, `run` enqueues the
// launches on m->hstream with device pointers into the staging buffer, and
// the outputs (laid out contiguously after the inputs) come back in one
// transfer.  in/out: host arrays and their sizes in 8-byte words (NULL arrays
// are skipped; their device pointer is NULL too).
struct HostArr {
  const void* host;
  int64_t words;
};
struct HostOut {
  void* host;
  int64_t words;      // staging space (whole 8-byte words)
  int64_t bytes = -1;  // bytes copied back (default: words * 8)
};
static inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// How a synchronous entry waits for its copy back (DRC_HOST_WAIT, in us): it
// polls the completion event for up to that long (default 300 us: one B = 1
// cycle is ~100 us, polling keeps the thread on its core instead of handing
// it to the scheduler and waking it up again), with a pause between polls,
// then blocks in hipEventSynchronize -- a long call (large B) does not hold a
// core busy for its whole GPU time.  0: block at once.
static int wait_done(drc_model* m) {
  static const int64_t spin_ns = 1000 * env_int("DRC_HOST_WAIT", 300, 0);
  if (hipEventRecord(m->hdone, m->hstream) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventRecord");
  if (spin_ns > 0) {
    const int64_t t_end = now_ns() + spin_ns;
    do {
      const hipError_t e = hipEventQuery(m->hdone);
      if (e == hipSuccess) return DRC_OK;
      if (e != hipErrorNotReady) return drc_amd::set_err(DRC_ERR_HIP, "hipEventQuery");
      for (int k = 0; k < 16; ++k) __builtin_ia32_pause();
    } while (now_ns() < t_end);
  }
  if (hipEventSynchronize(m->hdone) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventSynchronize");
  return DRC_OK;
}

template <class Run>
static int round_trip(drc_model* m, const HostArr* in, int nin, const HostOut* out, int nout, Run run) {
  const int64_t t0 = m->tl_on ? now_ns() : 0;
  int64_t wi = 0, wo = 0;
  for (int i = 0; i < nin; ++i) wi += in[i].host ? in[i].words : 0;
  for (int i = 0; i < nout; ++i) wo += out[i].host ? out[i].words : 0;
  if (int rc = ensure_staging(m, wi + wo)) return rc;
  double* dev = reinterpret_cast<double*>(m->stage);
  const void* din[16] = {nullptr};
  void* dout[16] = {nullptr};
  int64_t o = 0;
  for (int i = 0; i < nin; ++i)
    if (in[i].host) {
      std::memcpy(m->pinned + o, in[i].host, in[i].words * 8);
      din[i] = dev + o;
      o += in[i].words;
    }
  for (int i = 0; i < nout; ++i)
    if (out[i].host) {
      dout[i] = dev + o;
      o += out[i].words;
    }
  const int64_t t1 = m->tl_on ? now_ns() : 0;
  if (wi && hipMemcpyAsync(dev, m->pinned, wi * 8, hipMemcpyHostToDevice, m->hstream) != hipSuccess)
    return drc_amd::set_err(DRC_ERR_HIP, "hipMemcpyAsync H2D");
  if (int rc = run(din, dout)) return rc;
  if (wo && hipMemcpyAsync(m->pinned + wi, dev + wi, wo * 8, hipMemcpyDeviceToHost, m->hstream) != hipSuccess)
    return drc_amd::set_err(DRC_ERR_HIP, "hipMemcpyAsync D2H");
  const int64_t t2 = m->tl_on ? now_ns() : 0;
  if (int rc = wait_done(m)) return rc;
  const int64_t t3 = m->tl_on ? now_ns() : 0;
  o = wi;
  for (int i = 0; i < nout; ++i)
    if (out[i].host) {
      std::memcpy(out[i].host, m->pinned + o, out[i].bytes >= 0 ? out[i].bytes : out[i].words * 8);
      o += out[i].words;
    }
  if (m->tl_on) {
    const int64_t t4 = now_ns();
    for (int64_t v : {t0, t1, t2, t3, t4}) m->tl.push_back(v);
  }
  return DRC_OK;
}

static int host_call(drc_model* m, const drc_qpik_params* p, int stages, int64_t B, const HostIO& in,
                     double** outs, const int64_t* out_rows, int nouts, int32_t** iouts, int niouts,
                     uint64_t* stamps = nullptr /* host [kStamps][B]: the kernels' stage stamps */) {
  if (!m || !p) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  std::lock_guard<std::mutex> g(m->host_mu);
  if (hipSetDevice(m->device) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipSetDevice");
  HostArr ha[6];
  for (int i = 0; i < 6; ++i) ha[i] = {in.src[i], in.rows[i] * B};
  // outputs: the double arrays, the int32 arrays (one word per two), the stamps
  HostOut ho[8 + 2 + 1];
  int no = 0;
  for (int i = 0; i < nouts; ++i) ho[no++] = {outs[i], out_rows[i] * B};
  for (int i = 0; i < niouts; ++i) ho[no++] = {iouts[i], (B + 1) / 2, 4 * B};
  ho[no++] = {stamps, stamps ? drc_amd::kStamps * B : 0};
  auto run = [&](const void** din, void** dout) -> int {
    const double* d[6];
    for (int i = 0; i < 6; ++i) d[i] = static_cast<const double*>(din[i]);
    double* od[8] = {nullptr};
    for (int i = 0; i < nouts; ++i) od[i] = static_cast<double*>(dout[i]);
    int32_t* oi[2] = {nullptr, nullptr};
    for (int i = 0; i < niouts; ++i) oi[i] = static_cast<int32_t*>(dout[nouts + i]);
    uint64_t* ds = static_cast<uint64_t*>(dout[nouts + niouts]);
    if (ds && hipMemsetAsync(ds, 0, sizeof(uint64_t) * drc_amd::kStamps * B, m->hstream) != hipSuccess)
      return drc_amd::set_err(DRC_ERR_HIP, "hipMemsetAsync(stamps)");
    if (!stages)
      return drc_amd::launch(m, p, 0, B, d[0], d[1], d[2], d[3], d[4], d[5], od[0], oi[0], oi[1], nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, m->hstream, ds);
    return drc_amd::launch(m, p, 1, B, d[0], d[1], d[2], d[3], d[4], d[5], nullptr, nullptr, nullptr, od[0], od[1],
                           od[2], od[3], oi[0], od[4], m->hstream);
  };
  return round_trip(m, ha, 6, ho, no, run);
}
}  // namespace drc_amd

extern "C" {
using drc_amd::HostIO;
using drc_amd::host_call;

int drc_qpik_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                  int32_t* status, int32_t* iters) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (!out || !status) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out and status are required");
  const int64_t n = m->hm.dev.nv, a = m->hm.dev.kind == 1 ? m->hm.dev.n_arm + m->hm.dev.n_wheel : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[1] = {out};
  const int64_t rows[1] = {a};
  int32_t* iouts[2] = {status, iters};
  return host_call(m, p, 0, B, in, outs, rows, 1, iouts, 2);
}

int drc_qpik_host_timed(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                        const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                        int32_t* status, int32_t* iters, drc_time_duration* ts) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (!out || !status || !ts) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out, status and time_status are required");
  std::memset(ts, 0, sizeof(*ts));
  if (B <= 0) return B == 0 ? DRC_OK : drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  const int64_t n = m->hm.dev.nv, a = m->hm.dev.kind == 1 ? m->hm.dev.n_arm + m->hm.dev.n_wheel : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[1] = {out};
  const int64_t rows[1] = {a};
  int32_t* iouts[2] = {status, iters};
  std::vector<uint64_t> st(static_cast<size_t>(drc_amd::kStamps * B));
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = host_call(m, p, 0, B, in, outs, rows, 1, iouts, 2, st.data());
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc) return rc;
  // stamps are s_memrealtime ticks (100 MHz); per-instance stage durations, averaged
  // (the region was cleared before the launch: an instance whose stamps are
  // missing -- a debug task stage that does not stamp -- or out of order is
  // left out of the averages)
  const double tick = 1e-8;
  double task = 0, asmb = 0, solve = 0, store = 0, span = 0;
  int64_t valid = 0;
  for (int64_t b = 0; b < B; ++b) {
    auto at = [&](int k) { return st[static_cast<size_t>(k * B + b)]; };
    bool ok = at(0) != 0;
    for (int k = 1; k < drc_amd::kTimeStamps && ok; ++k) ok = at(k) >= at(k - 1);
    if (!ok) continue;
    auto dt = [&](int k1, int k0) { return static_cast<double>(at(k1) - at(k0)) * tick; };
    task += dt(drc_amd::ST_TASK1, drc_amd::ST_TASK0);
    asmb += dt(drc_amd::ST_ASM, drc_amd::ST_QP0);
    solve += dt(drc_amd::ST_SOLVED, drc_amd::ST_ASM);
    store += dt(drc_amd::ST_OUT, drc_amd::ST_SOLVED);
    span += dt(drc_amd::ST_OUT, drc_amd::ST_TASK0);
    ++valid;
  }
  if (valid == 0) {  // no stamps (a debug stage): the whole call counts as getSolution's place
    ts->solve_qp = wall;
    return DRC_OK;
  }
  const double inv = 1.0 / static_cast<double>(valid);
  ts->set_ineq = task * inv;         // FK, J, manipulability + gradient, min distance + gradient
  ts->set_constraint = asmb * inv;   // P, q, bounds, CBF rows stacked (QP_base.h:202-227)
  ts->set_qp = ts->set_ineq + ts->set_constraint;
  ts->set_solver = solve * inv;      // Ruiz scaling, factorisation, ADMM, certified polish
  // output store plus what the call spends outside the instance (launch,
  // transfers, synchronisation): getSolution's place in the reference
  ts->solve_qp = store * inv + (wall - span * inv > 0 ? wall - span * inv : 0.0);
  return DRC_OK;
}

int drc_debug_qpik_stamps(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                          const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                          int32_t* status, int32_t* iters, uint64_t* stamps) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (!out || !status || !stamps) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out, status and stamps are required");
  const int64_t n = m->hm.dev.nv, a = m->hm.dev.kind == 1 ? m->hm.dev.n_arm + m->hm.dev.n_wheel : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[1] = {out};
  const int64_t rows[1] = {a};
  int32_t* iouts[2] = {status, iters};
  return host_call(m, p, 0, B, in, outs, rows, 1, iouts, 2, stamps);
}

int drc_qpik_stages_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                         const double* xt, const double* xdt, const double* xi, const double* xdi, double* pose,
                         double* jac, double* man, double* dist, int32_t* pair, double* xdd) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const int64_t n = m->hm.dev.nv, na = m->hm.dev.kind == 1 ? m->hm.dev.n_arm : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[5] = {pose, jac, man, dist, xdd};
  const int64_t rows[5] = {12, 6 * n, 1 + na, 1 + n, 6};
  int32_t* iouts[1] = {pair};
  return host_call(m, p, 1, B, in, outs, rows, 5, iouts, 1);
}


// ---- per-cycle kinematics and state ----------------------
int drc_kinematics_batch(const drc_model* m, int frame_id, int64_t B, const double* q, const double* qdot,
                         double* pose, double* jac, double* xdot, void* stream) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  drc_qpik_params p;
  if (int rc = drc_default_qpik_params(m, 1, &p)) return rc;
  p.frame_id = frame_id;
  return drc_amd::launch_closed_form(m, &p, 3, B, q, qdot, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                     stream, pose, jac, xdot);
}

int drc_state_host(drc_model* m, int frame_id, int64_t B, const double* q, const double* qdot, double* pose,
                   double* jac, double* xdot, double* M, double* M_inv, double* g, double* nle, double* c) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!q) return set_err(DRC_ERR_INVALID_ARGUMENT, "q is required");
  if ((xdot || nle || c) && !qdot) return set_err(DRC_ERR_INVALID_ARGUMENT, "qdot is required for xdot / nle / c");
  const int64_t n = m->hm.dev.nv;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const drc_amd::HostArr in[2] = {{q, n * B}, {qdot, n * B}};
  const drc_amd::HostOut out[8] = {{pose, 12 * B}, {jac, 6 * n * B}, {xdot, 6 * B}, {M, n * n * B},
                                   {M_inv, n * n * B}, {g, n * B}, {nle, n * B}, {c, n * B}};
  auto run = [&](const void** din, void** dout) -> int {
    const double* dq = static_cast<const double*>(din[0]);
    const double* dqd = static_cast<const double*>(din[1]);
    double* o[8];
    for (int i = 0; i < 8; ++i) o[i] = static_cast<double*>(dout[i]);
    if (pose || jac || xdot)
      if (int rc = drc_kinematics_batch(m, frame_id, B, dq, dqd, o[0], o[1], o[2], m->hstream)) return rc;
    if (M || M_inv || g || nle || c)
      if (int rc = drc_dynamics_batch(m, 0, B, dq, dqd, o[3], o[4], o[5], o[6], o[7], m->hstream)) return rc;
    return DRC_OK;
  };
  return drc_amd::round_trip(m, in, 2, out, 8, run);
}

// ---- closed-form controllers ------------------------------
int drc_clik_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, const double* null_qdot,
                   double* qdot_out, void* stream) {
  return drc_amd::launch_closed_form(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, null_qdot, qdot_out, stream);
}

int drc_osf_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, const double* null_torque,
                  double* tau_out, void* stream) {
  return drc_amd::launch_closed_form(m, p, 2, B, q, qdot, xt, xdt, xi, xdi, null_torque, tau_out, stream);
}

int drc_closed_form_host(drc_model* m, const drc_qpik_params* p, int kind, int64_t B, const double* q,
                         const double* qdot, const double* xt, const double* xdt, const double* xi, const double* xdi,
                         const double* nullv, double* out) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (kind != 1 && kind != 2) return set_err(DRC_ERR_INVALID_ARGUMENT, "kind must be 1 (CLIK) or 2 (OSF)");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!out) return set_err(DRC_ERR_INVALID_ARGUMENT, "out is required");
  const int64_t n = m->hm.dev.nv;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[7] = {q, qdot, xt, xdt, xi, xdi, nullv};
  const int64_t rows[7] = {n, n, 12, 6, 12, 6, n};
  int64_t words = n * B;
  for (int i = 0; i < 7; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 7; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_amd::launch_closed_form(m, p, kind, B, din[0], din[1], din[2], din[3], din[4], din[5], din[6], dp,
                                       m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, dp, n * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

int drc_qpid_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, double* qdd, double* tau,
                  int32_t* status, int32_t* iters) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!qdd || !tau || !status) return set_err(DRC_ERR_INVALID_ARGUMENT, "qddot_out, tau_out and status are required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, na = d.kind == 1 ? d.n_arm + d.n_wheel : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[6] = {q, qdot, xt, xdt, xi, xdi};
  const int64_t rows[6] = {n, n, 12, 6, 12, 6};
  int64_t words = 2 * na * B + B;  // outputs + status/iters
  for (int i = 0; i < 6; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 6; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  double* dqdd = dp;
  double* dtau = dp + na * B;
  int32_t* dst = reinterpret_cast<int32_t*>(dp + 2 * na * B);
  int32_t* dit = iters ? dst + B : nullptr;
  int rc = drc_qpid_batch(m, p, B, din[0], din[1], din[2], din[3], din[4], din[5], dqdd, dtau, dst, dit, m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(qdd, dqdd, na * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipMemcpyAsync(tau, dtau, na * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipMemcpyAsync(status, dst, B * 4, hipMemcpyDeviceToHost, m->hstream));
  if (iters) HIP_TRY(hipMemcpyAsync(iters, dit, B * 4, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

// ---- joint-space dynamics ------------------------------
int drc_dynamics_batch(drc_model* m, int actuated, int64_t B, const double* q, const double* qdot, double* M,
                       double* M_inv, double* g, double* nle, double* c, void* stream) {
  using drc_amd::set_err;
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B < 0) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (!q) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "q is required");
  if ((nle || c) && !qdot) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot is required for nle / c");
  if (actuated && m->hm.dev.kind != 1)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "actuated dynamics need a mobile-manipulator model");
  if (B > 0x7ffffff0) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  HIP_TRY(hipSetDevice(m->device));
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  int* list = nullptr;
  drc_amd::StreamCtx* cx = nullptr;
  drc_amd::DoneGuard done_guard{cx, reinterpret_cast<hipStream_t>(stream)};
  if (M_inv) {
    std::lock_guard<std::mutex> lk(m->mu);
    if (int r = drc_amd::stream_ctx(m, reinterpret_cast<hipStream_t>(stream), &cx)) return r;
    if (cx->dyn_list_cap < B + 1) {
      if (cx->dyn_list) HIP_TRY(hipFree(cx->dyn_list));
      cx->dyn_list = nullptr;
      cx->dyn_list_cap = 0;
      HIP_TRY(hipMalloc(&cx->dyn_list, (B + 1) * sizeof(int)));
      cx->dyn_list_cap = B + 1;
    }
    list = cx->dyn_list;
  }
  const int rc = drc_amd::launch_dynamics(m->d_model, m->hm.dev, actuated != 0, B, q, qdot, M, M_inv, g, nle, c,
                                          list, reinterpret_cast<hipStream_t>(stream));
  if (rc == 1) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (rc) return drc_amd::set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  done_guard.ok = true;
  return DRC_OK;
}

int drc_dynamics_host(drc_model* m, int actuated, int64_t B, const double* q, const double* qdot, double* M,
                      double* M_inv, double* g, double* nle, double* c) {
  using drc_amd::set_err;
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B <= 0) return B == 0 ? DRC_OK : drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!q) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "q is required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, no = actuated ? d.n_arm + d.n_wheel : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  double* outs[5] = {M, M_inv, g, nle, c};
  const int64_t rows[5] = {no * no, no * no, no, no, no};
  int64_t words = (qdot ? 2 : 1) * n * B;
  for (int i = 0; i < 5; ++i) words += outs[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  double* dq = dp;
  dp += n * B;
  HIP_TRY(hipMemcpyAsync(dq, q, n * B * 8, hipMemcpyHostToDevice, m->hstream));
  double* dqd = nullptr;
  if (qdot) {
    dqd = dp;
    dp += n * B;
    HIP_TRY(hipMemcpyAsync(dqd, qdot, n * B * 8, hipMemcpyHostToDevice, m->hstream));
  }
  double* dout[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 5; ++i)
    if (outs[i]) {
      dout[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_dynamics_batch(m, actuated, B, dq, dqd, dout[0], dout[1], dout[2], dout[3], dout[4], m->hstream);
  if (rc) return rc;
  for (int i = 0; i < 5; ++i)
    if (outs[i]) HIP_TRY(hipMemcpyAsync(outs[i], dout[i], rows[i] * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

// ---- joint torque step ---------------------------------
int drc_joint_torque_step_batch(drc_model* m, int64_t B, const double* q, const double* qdot, const double* q_target,
                                const double* qdot_target, const double* qddot_target, double dt, const double* kp,
                                const double* kv, double* tau, void* stream) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (!q || !tau) return set_err(DRC_ERR_INVALID_ARGUMENT, "q and tau are required");
  if (!qddot_target && (!qdot || !qdot_target))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "qdot and qdot_target are required without qddot_target");
  const drc_amd::DevModel& d = m->hm.dev;
  const int nb = d.kind == 1 ? d.n_arm : d.nv;
  double kpv[drc_amd::kMaxJoints], kvv[drc_amd::kMaxJoints];
  for (int i = 0; i < nb; ++i) {  // robot_controller.cpp:14-15 (MoMa :17-18): 400 / 40
    kpv[i] = kp ? kp[i] : 400.0;
    kvv[i] = kv ? kv[i] : 40.0;
  }
  HIP_TRY(hipSetDevice(m->device));
  const int rc = drc_amd::launch_torque_step(m->d_model, d, B, q, qdot, q_target, qdot_target, qddot_target, dt, kpv,
                                             kvv, tau, reinterpret_cast<hipStream_t>(stream));
  if (rc == 1) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (rc) return set_err(DRC_ERR_HIP, std::string("torque step launch: ") + hipGetErrorString(hipGetLastError()));
  return DRC_OK;
}

int drc_joint_torque_step_host(drc_model* m, int64_t B, const double* q, const double* qdot, const double* q_target,
                               const double* qdot_target, const double* qddot_target, double dt, const double* kp,
                               const double* kv, double* tau) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!q || !tau) return set_err(DRC_ERR_INVALID_ARGUMENT, "q and tau are required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, nb = d.kind == 1 ? d.n_arm : d.nv;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[5] = {q, qdot, q_target, qdot_target, qddot_target};
  const int64_t rows[5] = {n, n, nb, nb, nb};
  int64_t words = nb * B;
  for (int i = 0; i < 5; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 5; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_joint_torque_step_batch(m, B, din[0], din[1], din[2], din[3], din[4], dt, kp, kv, dp, m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(tau, dp, nb * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

}  // extern "C"

