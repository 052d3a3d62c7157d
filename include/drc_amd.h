/*
 * drc_amd.h — C-ABI of the MI355X-native batched QP-IK solver.
 *
 * This is the drop-in boundary for the per-control-cycle hot path of
 * YoungWook0533/dyros_robot_controller.  Plain C: opaque
 * handles, plain pointers and sizes, integer return codes, no C++ types and
 * no exceptions cross it.  Every entry point names the reference interface
 * it replaces (file:line in the reference tree).
 *
 * Conventions
 *  - Batched arrays are structure-of-arrays, field-major: element (f, b) of
 *    a [F][B] array is at ptr[f * B + b].  All batched pointers are DEVICE
 *    pointers owned by the caller (HBM resident); `stream` is a hipStream_t
 *    (NULL = default stream).  Calls are asynchronous on that stream.  A
 *    model keeps its per-call scratch (task records, work-queue counters)
 *    per caller stream (at most 8 streams; see drc_model_release_stream), so
 *    calls on one model from several streams never share scratch, and calls
 *    from several host threads are safe (each call's launches are enqueued as
 *    a unit).  The internal fork/join streams of the concurrent sub-batches
 *    are per model, shared by the caller streams.
 *  - Poses are 12 doubles: R column-major (9) then p (3) — Eigen::Affine3d
 *    `linear()` memory order followed by `translation()`.
 *  - Velocities / twists are [v(3); w(3)] in the world frame
 *    (Pinocchio LOCAL_WORLD_ALIGNED, robot_data.cpp:401).
 *
 * Diagnostic entries with no reference counterpart (kernel timing, stage
 * stamps, LDS / occupancy plans, the lane-stage switch) are declared in
 * drc_amd_debug.h; the product boundary is this header.
 */
#ifndef DRC_AMD_H
#define DRC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ------------------------------------------------------ */
enum {
    DRC_OK = 0,
    DRC_ERR_INVALID_ARGUMENT = 1,
    DRC_ERR_FILE = 2,            /* URDF missing: reference std::exit()s (robot_data.cpp:17-18) */
    DRC_ERR_PARSE = 3,
    DRC_ERR_UNSUPPORTED = 4,     /* model outside the kernel's limits          */
    DRC_ERR_UNKNOWN_LINK = 5,    /* reference: stderr + zero result (:395-399) */
    DRC_ERR_HIP = 6,
    DRC_ERR_SIZE_MISMATCH = 7    /* reference: std::runtime_error (robot_controller.cpp:23-26) */
};

/* ---- per-instance solve status (mirrors OSQP status values) ------------ */
enum {
    DRC_STATUS_SOLVED = 1,
    DRC_STATUS_MAX_ITER = -2,
    DRC_STATUS_PRIMAL_INFEASIBLE = -3,
    DRC_STATUS_NONFINITE = -10
};

/* ---- controller entry points (robot_controller.h) ---------------------- */
enum {
    DRC_MODE_QPIK = 0,           /* QPIK(xdot_target)              manipulator/robot_controller.cpp:277 */
    DRC_MODE_QPIK_STEP = 1,      /* QPIKStep(x_target, xdot_target)                                :292 */
    DRC_MODE_QPIK_CUBIC = 2      /* QPIKCubic(x_t, xd_t, x_i, xd_i, t, t0, T)                     :303 */
};

/* ---- mobile base description (type_define.h:58-72 KinematicParam) ------ */
enum { DRC_DRIVE_DIFFERENTIAL = 0, DRC_DRIVE_MECANUM = 1, DRC_DRIVE_CASTER = 2 };
#define DRC_MAX_WHEELS 8
typedef struct drc_kinematic_param {
    int type;
    double wheel_radius;
    double max_lin_speed, max_ang_speed, max_lin_acc, max_ang_acc;
    double base_width;                              /* differential */
    int n_wheels;                                   /* mecanum wheels / casters (W = 2 per caster) */
    double roller_angles[DRC_MAX_WHEELS];
    double base2wheel_positions[DRC_MAX_WHEELS][2];
    double base2wheel_angles[DRC_MAX_WHEELS];
    double wheel_offset;                            /* caster */
} drc_kinematic_param;

/* type_define.h:151-156 / :167-171 */
typedef struct drc_joint_index { int virtual_start, mani_start, mobi_start; } drc_joint_index;
typedef struct drc_actuator_index { int mani_start, mobi_start; } drc_actuator_index;

/* ---- QP solver settings: OSQP's ADMM (QP_base.h:143-165) --------------- */
typedef struct drc_solver_settings {
    double rho, sigma, alpha;          /* 0.1, 1e-6, 1.6                    */
    double eps_abs, eps_rel;           /* 1e-3, 1e-3 (reference: defaults)  */
    double eps_prim_inf;               /* 1e-4                              */
    int max_iter;                      /* 4000                              */
    int check_termination;             /* 25                                */
    int scaling;                       /* 10 Ruiz iterations                */
    int adaptive_rho;                  /* 1                                 */
    int adaptive_rho_interval;         /* 25                                */
    double adaptive_rho_tolerance;     /* 5                                 */
    int polish;                        /* reference: 0                      */
    int polish_refine_iter;            /* 3                                 */
    double delta;                      /* 1e-6                              */
    int exact;                         /* 1: certified polish + tight fallback (parity mode) */
    double eps_exact;                  /* 1e-9 KKT acceptance of a polished point */
    double eps_fallback;               /* 1e-7 ADMM-only termination when polish keeps failing */
} drc_solver_settings;

/* ---- QPIK parameters (controller gains + QP constants) ----------------- */
typedef struct drc_qpik_params {
    double kp[6], kv[6];               /* manipulator: 100 / 20 (robot_controller.cpp:12-13)
                                          MoMa: 400 / 0 (mobile_manipulator/robot_controller.cpp:15) */
    double feedforward;                /* MoMa QPIKStep adds xdot_target (:177): 1; manipulator 0 */
    double alpha_cbf;                  /* 50      (QP_IK.cpp:101)           */
    double w_reg;                      /* 1.0 / 0.01 (QP_IK.cpp:81, MoMa :71) */
    double slack_w;                    /* 1000    (QP_IK.cpp:83-86)         */
    double man_min;                    /* 0.01    (QP_IK.cpp:122)           */
    double dist_min;                   /* 0.05    (QP_IK.cpp:130)           */
    int mode;                          /* DRC_MODE_*                        */
    int frame_id;                      /* from drc_model_find_frame         */
    double t, t0, duration;            /* QPIKCubic timing                  */
    drc_solver_settings solver;
} drc_qpik_params;

typedef struct drc_model drc_model;     /* opaque; owns its device copy */

/* Manipulator::RobotData(urdf, srdf, packages)  manipulator/robot_data.h:49,
 * robot_data.cpp:7-70 (model, collision pairs, limits).  `device` = HIP
 * device ordinal that receives the model constants. */
int drc_model_create_manipulator(const char* urdf_path, const char* srdf_path,
                                 const char* packages_path, int device, drc_model** out);

/* MobileManipulator::RobotData(param, joint_idx, actuator_idx, urdf, srdf, packages)
 * mobile_manipulator/robot_data.h:55, robot_data.cpp:7-44. */
int drc_model_create_mobile_manipulator(const drc_kinematic_param* param,
                                        const drc_joint_index* joint_idx,
                                        const drc_actuator_index* actuator_idx,
                                        const char* urdf_path, const char* srdf_path,
                                        const char* packages_path, int device, drc_model** out);

void drc_model_destroy(drc_model* model);

/* getDof / getActuatordDof / getManipulatorDof / getMobileDof
 * (manipulator/robot_data.h, mobile_manipulator/robot_data.h) and the
 * collision model size (geometries, active pairs). */
int drc_model_info(const drc_model* model, int* dof, int* actuated_dof, int* mani_dof,
                   int* mobi_dof, int* n_geoms, int* n_pairs);

/* getJointPositionLimit / getJointVelocityLimit (robot_data.h) — host arrays [dof] */
int drc_model_limits(const drc_model* model, double* q_lb, double* q_ub, double* qdot_lb,
                     double* qdot_ub);

/* pinocchio Model::getFrameId(link_name) as used by every getter
 * (robot_data.cpp:380,394): DRC_ERR_UNKNOWN_LINK when absent. */
int drc_model_find_frame(const drc_model* model, const char* link_name, int* frame_id);

/* Mobile FK Jacobian J_mobile (3 x W, row-major) of the base
 * (mobile/robot_data.cpp:123-176); host array.  Differential / mecanum only:
 * a caster base's J_mobile depends on the steer angles (drc_mobile_fk_jacobian). */
int drc_model_mobile_fk_jacobian(const drc_model* model, double* J3xW);

/* Mobile::RobotData::computeFKJacobian(wheel_pos) (mobile/robot_data.cpp:123-204)
 * for any drive, host arrays: J3xW [3][W] row-major; wheel_pos [W] (caster:
 * steer angle at 2i, drive angle at 2i+1; ignored otherwise, may be NULL);
 * *n_wheels receives W.  KinematicParam.n_wheels counts mecanum wheels or
 * casters (W = 2 x casters, :27-30). */
int drc_mobile_fk_jacobian(const drc_kinematic_param* param, const double* wheel_pos, double* J3xW, int* n_wheels);
/* Mobile::RobotController::computeIKJacobian (mobile/robot_controller.cpp:55-125):
 * wheel velocities = J [W][3] row-major * base twist; same arguments. */
int drc_mobile_ik_jacobian(const drc_kinematic_param* param, const double* wheel_pos, double* JWx3, int* n_wheels);

/* Reference defaults for the model kind (robot_controller ctor gains, QP
 * constants, OSQP defaults).  exact=0: the reference's OSQP settings
 * (eps 1e-3, no polish); exact=1: certified-optimal settings used for
 * parity. */
int drc_default_qpik_params(const drc_model* model, int exact, drc_qpik_params* params);

/* Batched QPIK / QPIKStep / QPIKCubic.
 *   Manipulator  (robot_controller.cpp:277-317): q, qdot [dof][B].
 *   Mobile manip (mobile_manipulator/robot_controller.cpp:147-197): q, qdot
 *       are the full joint vectors [dof][B] in JointIndex order
 *       (getJointVector, mobile_manipulator/robot_data.cpp:418-427).
 *   x_target [12][B] (modes STEP/CUBIC), xdot_target [6][B],
 *   x_init [12][B] / xdot_init [6][B] (mode CUBIC only, else NULL).
 *   qdot_out [na][B]: manipulator na = dof (QPIK returns qdot);
 *       MoMa na = actuated dof in ActuatorIndex order (eta, split into
 *       (qdot_mobile, qdot_arm) by ActuatorIndex, :161-164).
 *   status [B] (DRC_STATUS_*), iters [B] (may be NULL).
 * Non-solved instances get a zero output (QP_IK.cpp:56-61). */
int drc_qpik_batch(const drc_model* model, const drc_qpik_params* params, int64_t B,
                   const double* q, const double* qdot, const double* x_target,
                   const double* xdot_target, const double* x_init, const double* xdot_init,
                   double* qdot_out, int32_t* status, int32_t* iters, void* stream);

/* Stage outputs of the same kernel for parity checks: per instance
 *   pose [12][B]  (getPose with the pose at the current q — SURVEY Q1),
 *   jac  [6*dof][B] row-major (getJacobian, LWA),
 *   man  [1+mani][B] (manipulability, grad)  (getManipulability(true,false)),
 *   dist [1+dof][B]  (distance, grad)        (getMinDistance(true,false,false)),
 *   pair [B] (argmin collision pair), xdot_des [6][B] (the QP's task velocity).
 * Any output pointer may be NULL.  params->frame_id == -1 selects no task
 * frame (pose/jac/man/xdot_des then refer to the last joint's frame), for
 * callers that only need the distance stage (getMinDistance). */
int drc_qpik_stages_batch(const drc_model* model, const drc_qpik_params* params, int64_t B,
                          const double* q, const double* qdot, const double* x_target,
                          const double* xdot_target, const double* x_init,
                          const double* xdot_init, double* pose, double* jac, double* man,
                          double* dist, int32_t* pair, double* xdot_des, void* stream);

/* Host-buffer forms of drc_qpik_batch / drc_qpik_stages_batch: same
 * arguments, but every array is a HOST array ([field][B], row stride B).  The
 * call stages them through model-owned device memory on an internal stream
 * and returns when the outputs are back on the host (PCIe-inclusive).  Calls
 * on one model are serialised.  Used by the C++ facade (include/drc_amd.hpp)
 * for the reference's single-robot signatures (B = 1). */
int drc_qpik_host(drc_model* model, const drc_qpik_params* params, int64_t B,
                  const double* q, const double* qdot, const double* x_target,
                  const double* xdot_target, const double* x_init, const double* xdot_init,
                  double* qdot_out, int32_t* status, int32_t* iters);
int drc_qpik_stages_host(drc_model* model, const drc_qpik_params* params, int64_t B,
                         const double* q, const double* qdot, const double* x_target,
                         const double* xdot_target, const double* x_init,
                         const double* xdot_init, double* pose, double* jac, double* man,
                         double* dist, int32_t* pair, double* xdot_des);

/* QP::TimeDuration (include/dyros_robot_controller/QP_base.h:19-43): seconds
 * per stage of one solve, as QPBase::solveQP fills it (:100-174). */
typedef struct drc_time_duration {
    double set_qp;          /* set_cost + set_bound + set_ineq + set_eq + set_constraint */
    double set_cost, set_bound, set_ineq, set_eq, set_constraint;
    double set_solver;      /* OSQP setup + solve (QP_base.h:143-170) */
    double solve_qp;        /* getSolution (:172-174) */
} drc_time_duration;

/* drc_qpik_host with QP::TimeDuration filled from per-instance stage stamps
 * the kernels write (s_memrealtime, averaged over the B instances):
 *   set_ineq       the task stage: FK, J, manipulability and its gradient, min
 *                  self-distance and its gradient (what setCost / setIneqConstraint
 *                  query, QP_IK.cpp:69-131, done in one pass);
 *   set_constraint assembly of P, q, bounds and the CBF rows (QP_base.h:202-227);
 *   set_cost, set_bound, set_eq  0 (assembled in the passes above);
 *   set_qp         set_ineq + set_constraint;
 *   set_solver     Ruiz scaling, factorisation, ADMM and the certified polish;
 *   solve_qp       the output store plus the call's launch / transfer /
 *                  synchronisation time outside the instance.
 * Reference behaviour on failure (QP_IK.cpp:56-61, time_status.setZero()) is
 * the caller's: the C++ facade's QPIK::getOptJointVel zeroes it. */
int drc_qpik_host_timed(drc_model* model, const drc_qpik_params* params, int64_t B,
                        const double* q, const double* qdot, const double* x_target,
                        const double* xdot_target, const double* x_init, const double* xdot_init,
                        double* qdot_out, int32_t* status, int32_t* iters, drc_time_duration* time_status);

/* ---- per-cycle kinematics and robot state -----------
 * drc_kinematics_batch: getPose / getJacobian / getVelocity of one frame for B
 * robots (Manipulator::RobotData, src/manipulator/robot_data.cpp:378-422; the
 * pose at the current q) without the manipulability and
 * self-collision stages the QPIK path adds: pose [12][B], jac [6*dof][B]
 * row-major, xdot [6][B] = J qdot.  Any output may be NULL; qdot may be NULL
 * when xdot is.  frame_id from drc_model_find_frame (-1: the last joint).
 * Asynchronous on `stream`. */
int drc_kinematics_batch(const drc_model* model, int frame_id, int64_t B, const double* q,
                         const double* qdot, double* pose, double* jac, double* xdot, void* stream);
/* One control cycle's robot state for host arrays in ONE round trip: the
 * frame's pose / J / J qdot (drc_kinematics_batch) and updateDynamics' M,
 * M_inv, g, nle, c ([n*n][B], [n][B] as drc_dynamics_batch, actuated = 0) --
 * what RobotData::updateState caches and the cycle's getPose / getVelocity /
 * getJacobian / moveJointTorqueStep read (robot_data.cpp:91-124,378-422,
 * robot_controller.cpp:115-125).  The inputs go over in one transfer and the
 * outputs come back in one; any output may be NULL.  Synchronous. */
int drc_state_host(drc_model* model, int frame_id, int64_t B, const double* q, const double* qdot,
                   double* pose, double* jac, double* xdot, double* M, double* M_inv, double* g,
                   double* nle, double* c);

/* Concurrency of drc_qpik_batch: the batch is split into up to `chunks`
 * contiguous sub-batches (each >= 4096 instances, >= 16384 when there are 4)
 * that run concurrently: the last on the caller's stream, the others on
 * internal streams forked from and joined back to it (default 4: 4 streams,
 * HIP's default hardware queues per process).  Results do not depend on it. */
int drc_set_concurrency(drc_model* model, int chunks);

/* Fused task + QP kernel for the QP shapes the library compiles (the bundled
 * FR3, UR5e, Husky-FR3, XLS-FR3 layouts) and batches of up to 16 384
 * instances (the DRC_FUSE_MAX environment variable overrides): 1 (default)
 * runs such a drc_qpik_batch call as one kernel whose
 * waves take an instance through the task stage and the QP before the next,
 * the task record kept in LDS; 0 always runs the task-kernel -> QP-kernel
 * pipeline (drc_set_concurrency sub-batches), as larger batches do.  Results
 * are bit-identical either way (the library is built with -ffp-contract=on:
 * every multiply-add rounds the same in both kernels), so an instance's
 * result depends neither on the batch size nor on this switch. */
int drc_set_fusion(drc_model* model, int enable);

/* Frees the per-stream scratch (task-record pool, work-queue counters) the
 * model keeps for `stream`, after the stream's queued work has finished; call
 * it before destroying a stream the model was used on.  A model keeps at most
 * 8 such contexts in any case (the least recently used one is freed when a
 * ninth stream appears), so a caller cycling through streams cannot grow it
 * without bound.  No-op for a stream the model has not seen.  (Reference: no
 * counterpart — the reference's OSQP solver object is per controller.) */
int drc_model_release_stream(drc_model* model, void* stream);

const char* drc_error_string(int code);
/* Identity of this library build: a hash of its sources and compile flags
 * (build.sh).  Profiles measured on a build carry its id, so a counter
 * summary is only ever attributed to the build it came from.  (Reference: no
 * counterpart.) */
const char* drc_build_id(void);
/* Thread-local detail of the last failing call (parse position, HIP error). */
const char* drc_last_error(void);

/* ---- joint-space dynamics --------------------
 * drc_dynamics_batch: for B robots, the quantities RobotData::updateState caches
 * after updateDynamics:
 *   actuated = 0:  Manipulator::RobotData::updateDynamics (src/manipulator/robot_data.cpp:109-124)
 *                  M = crba (symmetric), M_inv = DyrosMath::PinvCOD(M), g = computeGeneralizedGravity,
 *                  nle = nonLinearEffects, c = nle - g;  n = dof.  Getters getMassMatrix / getMassMatrixInv /
 *                  getGravity / getNonlinearEffects / getCoriolis (robot_data.h:176-198); computeMassMatrix /
 *                  computeGravity / computeCoriolis / computeNonlinearEffects (robot_data.h:70-92) are the
 *                  same call with the fields they return.
 *   actuated = 1:  MobileManipulator::RobotData::updateDynamics (src/mobile_manipulator/robot_data.cpp:126-144)
 *                  S^T M S, PinvCOD(S^T M S), S^T g, S^T nle, S^T (nle - g) with the selection matrix of
 *                  robot_data.cpp:22-25,115-120;  n = actuated dof.  (getMassMatrixActuated etc.,
 *                  mobile_manipulator/robot_data.h:425-445; compute*Actuated :151-187.)
 * q, qdot: [dof][B] full joint vectors (JointIndex order for mobile manipulators); qdot may be NULL when
 * nle and c are NULL (treated as zero).  Outputs, any of which may be NULL: M, M_inv [n*n][B] (entry (i,j) at
 * field i*n + j), g, nle, c [n][B].  Gravity is Pinocchio's default (0, 0, -9.81).  Asynchronous on `stream`;
 * a second, usually empty, launch re-solves M_inv by a serial COD where the kernel cannot certify full rank. */
int drc_dynamics_batch(drc_model* model, int actuated, int64_t B, const double* q, const double* qdot,
                       double* M, double* M_inv, double* g, double* nle, double* c, void* stream);
/* Same contract with HOST buffers; synchronous (PCIe-inclusive). */
int drc_dynamics_host(drc_model* model, int actuated, int64_t B, const double* q, const double* qdot,
                      double* M, double* M_inv, double* g, double* nle, double* c);

/* ---- joint torque step ------------------------
 * Manipulator::RobotController::moveJointTorqueStep (src/manipulator/robot_controller.cpp:115-125) for B
 * robots, computing M and g in the same launch (robot_data.cpp:111-112):
 *   tau = M qddot_target + g                                     when qddot_target != NULL
 *   tau = M (kp .* (q_target - q) + kv .* (qdot_target - qdot)) + g   otherwise,
 * with q_target == NULL meaning q + dt * qdot_target: the Euler step that follows QPIK in the reference's
 * FR3 control loop (examples/C++/src/fr3_controller.cpp:132-134), so
 *   drc_qpik_batch(...qdot_out...) ; drc_joint_torque_step_batch(..., NULL, qdot_out, NULL, dt, ...)
 * is that whole cycle on the device.  Mobile manipulators: the arm block, as
 * MobileManipulator::RobotController::moveManipulatorJointTorqueStep (mobile_manipulator/robot_controller.cpp:103-118).
 * q, qdot: [dof][B]; q_target, qdot_target, qddot_target, tau: [nb][B] with nb = dof (manipulator) or the arm
 * dof (mobile manipulator).  kp, kv: HOST arrays [nb] or NULL for the reference defaults 400 / 40
 * (robot_controller.cpp:14-15). */
int drc_joint_torque_step_batch(drc_model* model, int64_t B, const double* q, const double* qdot,
                                const double* q_target, const double* qdot_target, const double* qddot_target,
                                double dt, const double* kp, const double* kv, double* tau, void* stream);
/* Same contract with HOST buffers; synchronous. */
int drc_joint_torque_step_host(drc_model* model, int64_t B, const double* q, const double* qdot,
                               const double* q_target, const double* qdot_target, const double* qddot_target,
                               double dt, const double* kp, const double* kv, double* tau);

/* ---- QPID: the torque-level QP ----------------------
 * Manipulator::RobotController::QPID / QPIDStep / QPIDCubic (src/manipulator/robot_controller.cpp:319-361) over
 * Manipulator::QPID (src/manipulator/QP_ID.cpp:7-193), and the MobileManipulator twins
 * (src/mobile_manipulator/robot_controller.cpp:199-250, QP_ID.cpp:7-184), for B robots.  Same params struct
 * as QPIK: mode DRC_MODE_QPID* (0 = QPID(xddot_target) with the task acceleration in xdot_target,
 * 1 = QPIDStep, 2 = QPIDCubic), kp/kv the task gains (defaults 100/20, MoMa 400/40).  Per call: M and g of the
 * equality rows are computed on the device (drc_dynamics_batch's kernel), then the QPID stage data (frame
 * Jacobian time variation, grad_dot terms of the singularity and self-collision CBF rows) and the QP.
 *   qddot_out [na][B]: qddot (manipulator) / eta_dot in ActuatorIndex order (MoMa);
 *   tau_out   [na][B]: joint torques / actuated torques;
 *   status [B], iters [B] (may be NULL).
 * Non-Solved: qddot = 0, tau = getGravity() (robot_controller.cpp:333-336); MoMa: tau[i] = the joint-order
 * getGravity()[i] — the reference slices that vector at ActuatorIndex offsets (mobile_manipulator/
 * robot_controller.cpp:211,218), restated as written. */
enum { DRC_MODE_QPID = 0, DRC_MODE_QPID_STEP = 1, DRC_MODE_QPID_CUBIC = 2 };
int drc_default_qpid_params(const drc_model* model, int exact, drc_qpik_params* params);
int drc_qpid_batch(const drc_model* model, const drc_qpik_params* params, int64_t B,
                   const double* q, const double* qdot, const double* x_target,
                   const double* xdot_target, const double* x_init, const double* xdot_init,
                   double* qddot_out, double* tau_out, int32_t* status, int32_t* iters, void* stream);
/* Stage outputs of the QPID task stage: as drc_qpik_stages_batch (xddot_des = the QP's task
 * acceleration), plus jdot [6*dof][B] (getJacobianTimeVariation, LWA, robot_data.cpp:404-417),
 * qpid_terms [8][B] = (Jdot v (6) with v = qdot or S eta, grad_dot_m . qdot_arm, grad_dot_d . qdot_arm) and
 * graddot [mani + dof][B] = the grad_dot vectors of getManipulability(true, true) (robot_data.cpp:555-569;
 * MoMa :477-492) and getMinDistance(true, true) (:496-512).  Any output may be NULL. */
int drc_qpid_stages_batch(const drc_model* model, const drc_qpik_params* params, int64_t B,
                          const double* q, const double* qdot, const double* x_target,
                          const double* xdot_target, const double* x_init, const double* xdot_init,
                          double* pose, double* jac, double* man, double* dist, int32_t* pair,
                          double* xddot_des, double* jdot, double* qpid_terms, double* graddot, void* stream);
int drc_qpid_stages_host(drc_model* model, const drc_qpik_params* params, int64_t B,
                         const double* q, const double* qdot, const double* x_target,
                         const double* xdot_target, const double* x_init, const double* xdot_init,
                         double* pose, double* jac, double* man, double* dist, int32_t* pair,
                         double* xddot_des, double* jdot, double* qpid_terms, double* graddot);
/* Host-buffer form of drc_qpid_batch (synchronous, PCIe-inclusive). */
int drc_qpid_host(drc_model* model, const drc_qpik_params* params, int64_t B,
                  const double* q, const double* qdot, const double* x_target,
                  const double* xdot_target, const double* x_init, const double* xdot_init,
                  double* qddot_out, double* tau_out, int32_t* status, int32_t* iters);

/* ---- closed-form controllers -------------------------
 * Manipulator::RobotController::CLIKStep / CLIKCubic (src/manipulator/robot_controller.cpp:156-214):
 *   qdot = J^+ (Kp e + xdot_target) + (I - J^+ J) null_qdot,  J^+ = DyrosMath::PinvCOD(J);
 *   params->mode DRC_MODE_QPIK_STEP (1) or DRC_MODE_QPIK_CUBIC (2); kp = Kp_task_ (kv is not used).
 * Manipulator::RobotController::OSF / OSFStep / OSFCubic (:216-275):
 *   Lambda = PinvCOD(J M^-1 J^T), tau = J^T Lambda xddot + (I - J^T Lambda J M^-1) null_torque + g,
 *   xddot = xdot_target (mode 0, OSF(xddot_target)) or Kp e + Kv (xdot_target - J qdot) (modes 1, 2);
 *   M^-1 = getMassMatrixInv, g = getGravity computed on the device in the same call.
 * Manipulator models only.  q, qdot [dof][B]; x_target [12][B]; xdot_target [6][B]; x_init/xdot_init for the
 * cubic forms; null_qdot / null_torque [dof][B] or NULL (the overloads without them); out [dof][B].
 * Parameters: drc_default_qpik_params (Kp_task_ = 100, Kv_task_ = 20). */
int drc_clik_batch(const drc_model* model, const drc_qpik_params* params, int64_t B, const double* q,
                   const double* qdot, const double* x_target, const double* xdot_target, const double* x_init,
                   const double* xdot_init, const double* null_qdot, double* qdot_out, void* stream);
int drc_osf_batch(const drc_model* model, const drc_qpik_params* params, int64_t B, const double* q,
                  const double* qdot, const double* x_target, const double* xdot_target, const double* x_init,
                  const double* xdot_init, const double* null_torque, double* tau_out, void* stream);
/* Host-buffer form of both (kind 1 = CLIK, 2 = OSF); synchronous. */
int drc_closed_form_host(drc_model* model, const drc_qpik_params* params, int kind, int64_t B, const double* q,
                         const double* qdot, const double* x_target, const double* xdot_target,
                         const double* x_init, const double* xdot_init, const double* null_vec, double* out);

#ifdef __cplusplus
}
#endif
#endif /* DRC_AMD_H */
