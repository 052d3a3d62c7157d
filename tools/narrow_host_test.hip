// Host-side harness for the device narrow-phase code (compiled for the CPU,
// no GPU needed): reads "type T(12) prm(3)" pairs on stdin, prints
// d pA pB lb cut_pruned, then the D17-refined d pA pB and whether the refinement
// was accepted: the kernels' per-pair rule (sphere closed forms,
// side-to-side cylinder closed form, else GJK / EPA), the broad-phase lower
// bound pair_lower_bound, and whether GJK's early exit fires with a cut just
// above the distance (it must not: its bound v.w/|v| never exceeds it).  Used by tests/test_narrow_host.py to check
// qpik_device.hpp against the oracle's shape_distance.
#include <cmath>
#include <cstdio>
#include "../dyros_robot_controller_amd/csrc/qpik_device.hpp"
using namespace drc_amd;
int main() {
  static EpaPoly ws;
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
    if (ta == kSphere || tb == kSphere) {
      d = sphere_pair(A, B, &pA, &pB);
    } else if (ta == kCylinder && tb == kCylinder && cyl_cyl_side(A, B, &d, &pA, &pB)) {
    } else {
      const GjkDist g = gjk(A, B);
      if (g.intersect) {
        d = epa_serial(A, B, &ws);
        pA = ld3(ws.out);
        pB = ld3(ws.out + 3);
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
    printf("%.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d\n", d,
           pA.x, pA.y, pA.z, pB.x, pB.y, pB.z, lb, pruned, dr, rA.x, rA.y, rA.z, rB.x, rB.y, rB.z, refined);
  }
}
