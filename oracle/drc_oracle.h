/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference QP-IK hot path
 * (YoungWook0533/dyros_robot_controller v0.3.0), used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker
 * and the CPU baseline.  It is never linked into, or called by, the product
 * library (dyros_robot_controller_amd/libdrc_amd.so).
 *
 * What it restates (file:line in the reference):
 *   kinematics       src/manipulator/robot_data.cpp:101-107,378-422
 *   manipulability   src/manipulator/robot_data.cpp:519-553
 *   min distance     src/manipulator/robot_data.cpp:424-494 (hpp-fcl GJK/EPA
 *                    semantics restated: parity unpinned)
 *   task helpers     include/math_type_define.h:62-298,563-570,633-687
 *   QP assembly      src/manipulator/QP_IK.cpp:7-131,
 *                    src/mobile_manipulator/QP_IK.cpp:7-128,
 *                    include/dyros_robot_controller/QP_base.h:65-227
 *   QP solve         QP_base.h:100-180 -> OSQP's ADMM (Stellato et al. 2020)
 *                    restated: Ruiz scaling, rho vector, adaptive rho,
 *                    termination, primal-infeasibility test and polish
 *   controllers      src/manipulator/robot_controller.cpp:277-317,
 *                    src/mobile_manipulator/robot_controller.cpp:147-197
 *   mobile FK Jac.   src/mobile/robot_data.cpp:138-176,
 *                    src/mobile_manipulator/robot_data.cpp:107-124
 */
#ifndef DRC_ORACLE_H
#define DRC_ORACLE_H
#include <stdint.h>

#define ORC_MAXJ 32
#define ORC_MAXG 96
#define ORC_MAXP 1024
#define ORC_MAXX 64
#define ORC_MAXC 128

typedef struct OracleModel {
    int nv;                          /* number of 1-DoF joints              */
    int parent[ORC_MAXJ + 1];        /* joint parent (0 = universe)         */
    int jtype[ORC_MAXJ + 1];         /* 0 revolute, 1 prismatic             */
    double jplace[ORC_MAXJ + 1][12]; /* R (row-major 9) + p (3), in parent  */
    double axis[ORC_MAXJ + 1][3];
    double lower[ORC_MAXJ], upper[ORC_MAXJ], vel[ORC_MAXJ];
    int ee_joint;                    /* task frame parent joint             */
    double ee_place[12];
    int ngeom;
    int gparent[ORC_MAXG];
    int gtype[ORC_MAXG];             /* 0 sphere, 1 cylinder, 2 box         */
    double gplace[ORC_MAXG][12];
    double gparam[ORC_MAXG][3];      /* sphere r | cyl r,h/2 | box half ext */
    int npairs;
    int pair_a[ORC_MAXP], pair_b[ORC_MAXP];
    /* whole-body (mobile manipulator) description; kind 0 = manipulator */
    int kind;                        /* 0 manipulator, 1 mobile manipulator */
    int n_arm, n_wheel;              /* MoMa: arm dof, wheel count          */
    int virtual_start, mani_start, mobi_start;   /* JointIndex            */
    int act_mani_start, act_mobi_start;          /* ActuatorIndex         */
    double J_mobile[3][8];           /* base twist / wheel velocity (3xW)   */
    int drive;                       /* 0 differential, 1 mecanum, 2 caster  */
    double wheel_radius, wheel_offset;
    double caster_pos[4][2];         /* caster: base2wheel_positions; J_mobile
                                      * then follows the steer angles       */
} OracleModel;

typedef struct OracleSettings {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf;
    int max_iter, check_termination, scaling;
    int adaptive_rho, adaptive_rho_interval;
    double adaptive_rho_tolerance;
    int polish, polish_refine_iter;
    double delta;
    int exact;                       /* certified polish + tight fallback   */
    double eps_exact;                /* strict KKT acceptance               */
    double eps_fallback;             /* ADMM-only tight termination         */
    int polish_cap;                  /* max reduced-KKT size (free variables
                                      * + active G rows), 0 = none; the
                                      * kernel's QPID buffers hold 48       */
    int polish_add_all;              /* infeasible polish point: add every
                                      * violated row (QPIK) or only the most
                                      * violated one (QPID)                 */
    int polish_guess;                /* first active-set guess: 0 OSQP's rule,
                                      * 1 projected Jacobi on the q-dot box
                                      * (polish_guess_jacobi), 2 that plus the
                                      * slack rule (polish_guess_slack; QPIK
                                      * parity mode) */
    int stop_at;                     /* > 0: stop at that ADMM iteration and
                                      * return its iterate as Solved (tests:
                                      * the other side's stopping point)    */
} OracleSettings;

typedef struct OracleParams {
    double kp[6], kv[6];
    double alpha_cbf, w_reg, slack_w, man_min, dist_min;
    int mode;                        /* 0 QPIK, 1 QPIKStep, 2 QPIKCubic     */
    double t, t0, duration;          /* QPIKCubic timing                    */
    OracleSettings solver;
} OracleParams;

/* per-instance diagnostics (stage parity) */
typedef struct OracleDiag {
    double pose[12];                 /* R row-major + p                    */
    double J[6 * ORC_MAXJ];          /* 6 x nv row-major                   */
    double xdot_des[6];
    double man, man_grad[ORC_MAXJ];
    double dist, dist_grad[ORC_MAXJ];
    int pair;
    int iters;
    int polished;
    /* QPID stage data (oracle_qpid_one) */
    double jdot_v[6];                /* Jdot * qdot (MoMa: Jdot * S * eta)  */
    double man_graddot[ORC_MAXJ];    /* getManipulability grad_dot (arm)    */
    double dist_graddot[ORC_MAXJ];   /* getMinDistance grad_dot (full dof)  */
    double man_gd, dist_gd;          /* grad_dot . qdot_arm used in the rows */
    double Jdot[6 * ORC_MAXJ];
    double res_ratio;                /* last termination check: max(pri/eps_pri, dua/eps_dua) */       /* frame Jacobian time variation        */
} OracleDiag;

enum { ORC_SOLVED = 1, ORC_MAX_ITER = -2, ORC_PRIMAL_INFEASIBLE = -3, ORC_NONFINITE = -10 };

void oracle_default_params(int kind, OracleParams* p, int exact);

/* One QPIK* solve (reference semantics) for one instance.
 * Manipulator: q, qdot[nv]; MoMa: q, qdot are the full joint vectors [nv].
 * x_target: 12 (R col-major 9, p 3); xdot_target: 6; for mode 2 also
 * x_init/xdot_init.  out: nv (manipulator) or A = n_wheel + n_arm (MoMa,
 * actuator order).  Returns status. */
int oracle_qpik_one(const OracleModel* m, const OracleParams* p,
                    const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target,
                    const double* x_init, const double* xdot_init,
                    double* out, OracleDiag* diag);

/* Batched SoA driver ([field][B] layout, the product's HBM layout) with a
 * pthread pool of nthreads workers.  Returns number of non-solved. */
int64_t oracle_qpik_batch(const OracleModel* m, const OracleParams* p, int64_t B,
                          const double* q, const double* qdot,
                          const double* x_target, const double* xdot_target,
                          const double* x_init, const double* xdot_init,
                          double* out, int32_t* status, int32_t* iters, int nthreads);
/* Same with stage data supplied (parity of the QP on identical data):
 * dist_in [1+nv][B] = (d, grad d) replaces getMinDistance's result, man_in
 * [1+narm][B] = (m, grad m) getManipulability's; NULL = computed. */
int64_t oracle_qpik_batch_dist(const OracleModel* m, const OracleParams* p, int64_t B,
                               const double* q, const double* qdot,
                               const double* x_target, const double* xdot_target,
                               const double* x_init, const double* xdot_init, const double* dist_in,
                               const double* man_in, double* out, int32_t* status, int32_t* iters, int nthreads);

/* QPID / QPIDStep / QPIDCubic for one instance (mode 0 takes the task
 * acceleration in xdot_target).  M, g: na x na (row-major) and na, the
 * matrices of the QP's equality rows (MoMa: S^T M S, S^T g); g_full: full
 * joint-order gravity (MoMa failure path).  Outputs qdd[na], tau[na]. */
void oracle_default_qpid_params(int kind, OracleParams* p, int exact);
int oracle_qpid_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target, const double* x_init,
                    const double* xdot_init, const double* M, const double* g, const double* g_full,
                    double* qdd, double* tau, OracleDiag* diag);
void oracle_qpid_stages(const OracleModel* m, const double* q, const double* qdot, double* Jdot,
                        double* man_graddot, double* dist_graddot);
void oracle_point_jacobian_dot(const OracleModel* m, const double* q, const double* qdot, int jid,
                               const double* p, double* J, double* Jdot);
void oracle_joint_placement(const OracleModel* m, const double* q, int jid, double* T12);

/* CLIKStep / CLIKCubic (mode 1 / 2) and OSF / OSFStep / OSFCubic (mode 0 / 1
 * / 2) of Manipulator::RobotController (robot_controller.cpp:156-275).
 * null_qdot / null_torque may be NULL (the overloads without them). */
void oracle_clik_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                     const double* x_target, const double* xdot_target, const double* x_init,
                     const double* xdot_init, const double* null_qdot, double* out);
void oracle_osf_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target, const double* x_init,
                    const double* xdot_init, const double* Minv, const double* g, const double* null_torque,
                    double* out);

void oracle_pinv_cod(const double* A, int m, int n, double* X);

/* stage helpers exposed for tests */
void oracle_fk_pose(const OracleModel* m, const double* q, double* pose12, double* J6xn);
void oracle_min_distance(const OracleModel* m, const double* q, double* dist, double* grad, int* pair);
void oracle_pair_distance(const OracleModel* m, const double* q, int pair, double* d, double* pA, double* pB);
void oracle_shape_distance(int ta, const double* TA, const double* prmA, int tb, const double* TB,
                           const double* prmB, double* d, double* pA, double* pB);
/* raw GJK / EPA results without the witness refinement (D17), for tests;
 * how: 0 closed form, 1 GJK, 2 EPA */
/* 1: getMinDistance's argmin by the kernel's pruned algorithm (closed forms,
 * lower bounds, GJK early exit, best-first EPA) instead of the reference's
 * all-pairs loop; same result.  Used by the FLOP count. */
void oracle_set_pruned_narrow_phase(int on);
void oracle_pair_distance_raw(const OracleModel* m, const double* q, int pair, double* d, double* pA, double* pB,
                              int* how);
void oracle_shape_distance_raw(int ta, const double* TA, const double* prmA, int tb, const double* TB,
                               const double* prmB, double* d, double* pA, double* pB, int* how);
void oracle_manipulability(const OracleModel* m, const double* q, double* man, double* grad);
int oracle_solve_qp(int nx, int nc, const double* P, const double* qv, const double* A,
                    const double* l, const double* u, const OracleSettings* s,
                    double* x, double* y, int* iters, int* polished);

#endif
