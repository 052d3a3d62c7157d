// Host-side harness for the device narrow-phase code (compiled for the CPU,
// no GPU needed): reads "type T(12) prm(3)" pairs on stdin, prints
// d pA pB lb cut_pruned wave_same: the kernels' per-pair rule (sphere closed forms,
// side-to-side cylinder closed form, else GJK / EPA), the broad-phase lower
// bound pair_lower_bound, and whether GJK's early exit fires with a cut just
// above the distance (it must not: its bound v.w/|v| never exceeds it).  Used by tests/test_narrow_host.py to check
// qpik_device.hpp against the oracle's shape_distance.
#include <cmath>
#include <cstdio>
#include "../dyros_robot_controller_amd/csrc/qpik_device.hpp"
using namespace drc_amd;
// the task kernel's wave form of an EPA step (epa_grow_walk on one lane, the
// new faces' geometry one per lane, epa_grow_finish), emulated serially
static void epa_step_wave(const Shape& A, const Shape& B, EpaPoly* E, int best) {
  const SV w = sup_md(A, B, ld3(E->fn[best]));
  bool stop = epa_gap_stop(E, best, w);
  for (int i = 0; !stop && i < E->nv; ++i) stop = epa_is_dup(E, i, w);
  if (stop) {
    E->stop = 1;
    return;
  }
  FaceMask vis{0, 0};
  for (int f = 0; f < E->nf; ++f)
    if (epa_sees(E, f, w.w)) vis.set(f);
  epa_grow_walk(E, w, best, vis);
  bool gfail = false;
  for (int i = 0; i < E->nnew; ++i) gfail |= !epa_face_geometry(E, E->newl[i], E->fd[best]);
  epa_grow_finish(E, best, gfail);
}
static double epa_wave(const Shape& A, const Shape& B, EpaPoly* E) {
  epa_init(A, B, E);
  for (int it = 0; it < 255 && !E->stop; ++it) epa_step_wave(A, B, E, epa_best_serial(E));
  return epa_finish(E, epa_best_serial(E));
}
int main() {
  static EpaPoly ws, ws2;
  int ta, tb;
  double TA[12], TB[12], pa[3], pb[3];
  while (scanf("%d", &ta) == 1) {
    for (double& v : TA) scanf("%lf", &v);
    for (double& v : pa) scanf("%lf", &v);
    scanf("%d", &tb);
    for (double& v : TB) scanf("%lf", &v);
    for (double& v : pb) scanf("%lf", &v);
    Shape A{ta, TA, pa[0], pa[1], pa[2]}, B{tb, TB, pb[0], pb[1], pb[2]};
    double d;
    V3 pA, pB;
    int wave_same = 1;  // EPA's wave form gives the serial form's result bit for bit
    if (ta == kSphere || tb == kSphere) {
      d = sphere_pair(A, B, &pA, &pB);
    } else if (ta == kCylinder && tb == kCylinder && cyl_cyl_side(A, B, &d, &pA, &pB)) {
    } else {
      const GjkDist g = gjk(A, B);
      if (g.intersect) {
        d = epa_serial(A, B, &ws);
        pA = ld3(ws.out);
        pB = ld3(ws.out + 3);
        const double d2 = epa_wave(A, B, &ws2);
        for (int i = 0; i < 6; ++i) wave_same &= ws.out[i] == ws2.out[i];
        wave_same &= d2 == d;
      } else {
        d = g.dist;
        pA = g.pA;
        pB = g.pB;
      }
    }
    // bounding radius of the swept core (model.cpp: sphere r, cylinder r,
    // box |half extents|)
    auto bound = [](int t, const double* p) {
      return t == kBox ? std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]) : p[0];
    };
    const double lb = (ta == kSphere || tb == kSphere) ? d : pair_lower_bound(A, B, bound(ta, pa), bound(tb, pb));
    int pruned = 0;
    if (ta != kSphere && tb != kSphere) {
      GjkState g;
      gjk_run(A, B, g, d + 1e-9 * (1 + std::fabs(d)));
      pruned = g.pruned;
    }
    // witness refinement of GJK / EPA results (D17)
    double dr = d;
    V3 rA = pA, rB = pB;
    int refined = 0;
    if (ta != kSphere && tb != kSphere && !(ta == kCylinder && tb == kCylinder && cyl_cyl_side(A, B, &dr, &rA, &rB))) {
      dr = d;
      refined = refine_witness(A, B, &dr, &rA, &rB) ? 1 : 0;
    }
    printf("%.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d\n", d,
           pA.x, pA.y, pA.z, pB.x, pB.y, pB.z, lb, pruned, wave_same, dr, rA.x, rA.y, rA.z, rB.x, rB.y, rB.z, refined);
  }
}
