// Host-side harness for the device narrow-phase code (compiled for the CPU,
// no GPU needed): reads "type T(12) prm(3)" pairs on stdin, prints d pA pB.
// Used by tests/test_narrow_host.py to check qpik_device.hpp against the
// oracle's shape_distance.
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
    printf("%.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", d, pA.x, pA.y, pA.z, pB.x, pB.y, pB.z);
  }
}
