"""MI355X-native batched QP-IK / whole-body QP-IK hot path of
YoungWook0533/dyros_robot_controller (drc/manipulator QPIK and
drc/mobile_manipulator QPIK), behind the reference's controller interface.

Product path: ``libdrc_amd.so`` (hand-written HIP for gfx950) through the
C-ABI in ``include/drc_amd.h``.  See DESIGN.md.
"""
import os

__version__ = "0.1.0"
PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROBOTS_DIR = os.path.join(PKG_DIR, "robots")


def robot_path(name, ext="urdf"):
    """Path of a bundled robot fixture, e.g. robot_path('fr3') -> .../fr3/fr3.urdf"""
    return os.path.join(ROBOTS_DIR, name, "%s.%s" % (name, ext))
