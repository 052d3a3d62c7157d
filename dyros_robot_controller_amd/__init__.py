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


# Bundled fixture robots (SURVEY.md §8 note N5): task link and, for the
# whole-body models, the mobile-base description the reference takes as
# KinematicParam / JointIndex / ActuatorIndex (type_define.h:58-171).
BUNDLED = {
    "fr3": dict(link="fr3_link8", kind="manipulator"),
    "ur5e": dict(link="tool0", kind="manipulator"),
    "husky_fr3": dict(link="fr3_link8", kind="mobile_manipulator", drive="differential", wheel_radius=0.165,
                      base_width=0.555, joint_index=(0, 3, 10), actuator_index=(0, 7)),
    "xls_fr3": dict(link="fr3_link8", kind="mobile_manipulator", drive="mecanum", wheel_radius=0.120,
                    roller_angles=[-0.7853981633974483, 0.7853981633974483, 0.7853981633974483,
                                   -0.7853981633974483],
                    base2wheel_positions=[(0.2225, 0.2045), (0.2225, -0.2045), (-0.2225, 0.2045),
                                          (-0.2225, -0.2045)],
                    base2wheel_angles=[0, 0, 0, 0], joint_index=(0, 3, 10), actuator_index=(0, 7)),
    "caster_fr3": dict(link="fr3_link8", kind="mobile_manipulator", drive="caster", wheel_radius=0.08,
                       wheel_offset=0.05, base2wheel_positions=[(0.25, 0.2), (-0.25, -0.2)],
                       joint_index=(0, 3, 10), actuator_index=(0, 7)),
}


def make_robot(name, device=None):
    """RobotData of a bundled robot (manipulator.RobotData or
    mobile_manipulator.RobotData) on ``device``."""
    spec = BUNDLED[name]
    if spec["kind"] == "manipulator":
        from .manipulator import RobotData
        return RobotData(robot_path(name), robot_path(name, "srdf"), device=device)
    from . import mobile_manipulator as MM
    drive = {"differential": MM.DriveType.Differential, "mecanum": MM.DriveType.Mecanum,
             "caster": MM.DriveType.Caster}[spec["drive"]]
    kp = MM.KinematicParam(drive, spec["wheel_radius"], base_width=spec.get("base_width"),
                           roller_angles=spec.get("roller_angles"),
                           base2wheel_positions=spec.get("base2wheel_positions"),
                           base2wheel_angles=spec.get("base2wheel_angles"), wheel_offset=spec.get("wheel_offset"))
    vs, ms, ws = spec["joint_index"]
    am, aw = spec["actuator_index"]
    return MM.RobotData(kp, MM.JointIndex(vs, ms, ws), MM.ActuatorIndex(am, aw), robot_path(name),
                        robot_path(name, "srdf"), device=device)
