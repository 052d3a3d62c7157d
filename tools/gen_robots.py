#!/usr/bin/env python3
"""Generate the robot model fixtures under dyros_robot_controller_amd/robots/.

Run in the build container only (it reads the reference's example FR3 model
once).  The outputs are *data fixtures*: a compact re-serialisation of the
FR3 kinematic/inertial/collision data (visual meshes, comments and ROS-only
tags dropped) and three authored models the reference does not ship
(SURVEY.md §8 note N5):

* ``ur5e``      — 6-DoF arm authored from the public UR5e kinematic and mass
                  data, with primitive (sphere/cylinder) collision bodies.
* ``husky_fr3`` — differential-drive base (2 wheels) + FR3, whole-body model
                  with 3 virtual joints (x, y, yaw), SURVEY.md §7 step 0.
* ``xls_fr3``   — 4-wheel mecanum base (Summit-XLS wheel geometry from
                  ``examples/C++/src/xls_controller.cpp:16-30``) + FR3.
* ``caster_fr3`` — base on two powered casters (steer + drive joint each,
                  DriveType::Caster, src/mobile/robot_data.cpp:179-204) + FR3.

Joint naming of the mobile models is chosen so that the Pinocchio/urdfdom
depth-first, name-sorted traversal yields [virtual(3) | arm(7) | wheels(W)],
i.e. JointIndex{virtual_start=0, mani_start=3, mobi_start=10} and
ActuatorIndex{mani_start=0, mobi_start=7}.
"""
import math
import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "dyros_robot_controller_amd", "robots")
REF_FR3 = "/root/reference/examples/robots/fr3"


def f(x):
    return repr(float(x)) if not isinstance(x, str) else x


def vec(v):
    return " ".join(f(x) for x in v)


class UrdfWriter:
    def __init__(self, name):
        self.name = name
        self.lines = []

    def link(self, name, inertial=None, collisions=()):
        if inertial is None and not collisions:
            self.lines.append(f'  <link name="{name}"/>')
            return
        self.lines.append(f'  <link name="{name}">')
        for (xyz, rpy, geom) in collisions:
            kind, dims = geom
            if kind == "sphere":
                g = f'<sphere radius="{f(dims[0])}"/>'
            elif kind == "cylinder":
                g = f'<cylinder radius="{f(dims[0])}" length="{f(dims[1])}"/>'
            else:
                g = f'<box size="{vec(dims)}"/>'
            self.lines.append(f'    <collision><origin xyz="{vec(xyz)}" rpy="{vec(rpy)}"/><geometry>{g}</geometry></collision>')
        if inertial is not None:
            mass, com, I = inertial
            self.lines.append(
                f'    <inertial><origin xyz="{vec(com)}" rpy="0 0 0"/><mass value="{f(mass)}"/>'
                f'<inertia ixx="{f(I[0])}" ixy="{f(I[1])}" ixz="{f(I[2])}" iyy="{f(I[3])}" iyz="{f(I[4])}" izz="{f(I[5])}"/></inertial>')
        self.lines.append("  </link>")

    def joint(self, name, jtype, parent, child, xyz, rpy, axis=None, limit=None):
        s = f'  <joint name="{name}" type="{jtype}"><parent link="{parent}"/><child link="{child}"/><origin xyz="{vec(xyz)}" rpy="{vec(rpy)}"/>'
        if axis is not None:
            s += f'<axis xyz="{vec(axis)}"/>'
        if limit is not None:
            lo, hi, vel, eff = limit
            s += f'<limit lower="{f(lo)}" upper="{f(hi)}" velocity="{f(vel)}" effort="{f(eff)}"/>'
        s += "</joint>"
        self.lines.append(s)

    def text(self):
        return "<?xml version=\"1.0\"?>\n<robot name=\"%s\">\n%s\n</robot>\n" % (self.name, "\n".join(self.lines))


def write_srdf(path, name, pairs):
    body = "\n".join(f'  <disable_collisions link1="{a}" link2="{b}" reason="{r}"/>' for a, b, r in pairs)
    with open(path, "w") as fh:
        fh.write(f'<?xml version="1.0"?>\n<robot name="{name}">\n{body}\n</robot>\n')


def _floats(s, n=None):
    v = [float(x) for x in s.split()]
    if n is not None:
        assert len(v) == n
    return v


def read_reference_fr3():
    """Pull links/joints/collisions/inertials out of the reference FR3 URDF."""
    tree = ET.parse(os.path.join(REF_FR3, "fr3.urdf"))
    root = tree.getroot()
    links, joints = {}, []
    for ln in root.findall("link"):
        cols = []
        for c in ln.findall("collision"):
            o = c.find("origin")
            xyz = _floats(o.get("xyz", "0 0 0"), 3) if o is not None else [0, 0, 0]
            rpy = _floats(o.get("rpy", "0 0 0"), 3) if o is not None else [0, 0, 0]
            g = c.find("geometry")[0]
            if g.tag == "sphere":
                geom = ("sphere", [float(g.get("radius"))])
            elif g.tag == "cylinder":
                geom = ("cylinder", [float(g.get("radius")), float(g.get("length"))])
            else:
                geom = ("box", _floats(g.get("size"), 3))
            cols.append((xyz, rpy, geom))
        inertial = None
        ie = ln.find("inertial")
        if ie is not None:
            o = ie.find("origin")
            com = _floats(o.get("xyz"), 3)
            m = float(ie.find("mass").get("value"))
            it = ie.find("inertia")
            I = [float(it.get(k)) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")]
            inertial = (m, com, I)
        links[ln.get("name")] = (inertial, cols)
    for j in root.findall("joint"):
        o = j.find("origin")
        ax = j.find("axis")
        lim = j.find("limit")
        joints.append(dict(
            name=j.get("name"), type=j.get("type"),
            parent=j.find("parent").get("link"), child=j.find("child").get("link"),
            xyz=_floats(o.get("xyz"), 3), rpy=_floats(o.get("rpy"), 3),
            axis=_floats(ax.get("xyz"), 3) if ax is not None else None,
            limit=(float(lim.get("lower")), float(lim.get("upper")), float(lim.get("velocity")),
                   float(lim.get("effort"))) if lim is not None else None))
    srdf = ET.parse(os.path.join(REF_FR3, "fr3.srdf")).getroot()
    disabled = [(d.get("link1"), d.get("link2"), d.get("reason")) for d in srdf.findall("disable_collisions")]
    return links, joints, disabled


def emit_fr3_arm(w, links, joints, mount_parent=None, mount_xyz=(0, 0, 0), skip_base=False):
    """Emit FR3 links and joints.  With mount_parent, fr3_link0 is attached to
    mount_parent through a fixed joint named ``fr3_mount_joint``."""
    order = ["fr3_link%d" % i for i in range(9)]
    if not skip_base:
        w.link("base_link")
    for ln in order:
        inertial, cols = links[ln]
        w.link(ln, inertial, cols)
    for j in joints:
        if j["name"] == "fr3_base_joint":
            if mount_parent is None:
                w.joint(j["name"], "fixed", j["parent"], j["child"], j["xyz"], j["rpy"])
            else:
                w.joint("fr3_mount_joint", "fixed", mount_parent, "fr3_link0", mount_xyz, (0, 0, 0))
            continue
        w.joint(j["name"], j["type"], j["parent"], j["child"], j["xyz"], j["rpy"], j["axis"], j["limit"])


def gen_fr3(links, joints, disabled):
    d = os.path.join(OUT, "fr3")
    os.makedirs(d, exist_ok=True)
    w = UrdfWriter("fr3")
    emit_fr3_arm(w, links, joints)
    with open(os.path.join(d, "fr3.urdf"), "w") as fh:
        fh.write(w.text())
    write_srdf(os.path.join(d, "fr3.srdf"), "fr3", disabled)


def cyl_inertia(m, r, h):
    ixx = m * (3 * r * r + h * h) / 12.0
    return [ixx, 0.0, 0.0, ixx, 0.0, 0.5 * m * r * r]


def gen_ur5e():
    """UR5e: public kinematic data (d1 0.1625, a2 -0.425, a3 -0.3922,
    d4 0.1333, d5 0.0997, d6 0.0996) and link masses; collision primitives
    authored to wrap the published link envelopes."""
    d = os.path.join(OUT, "ur5e")
    os.makedirs(d, exist_ok=True)
    h = math.pi / 2
    pi = math.pi
    w = UrdfWriter("ur5e")
    w.link("world")
    w.link("base_link", (4.0, [0, 0, 0.05], cyl_inertia(4.0, 0.075, 0.1)),
           [([0, 0, 0.05], [0, 0, 0], ("cylinder", [0.076, 0.1])),
            ([0, 0, 0.10], [0, 0, 0], ("sphere", [0.07]))])
    w.link("shoulder_link", (3.761, [0, 0, 0], cyl_inertia(3.761, 0.06, 0.15)),
           [([0, 0, 0], [0, 0, 0], ("cylinder", [0.062, 0.14])),
            ([0, 0, 0.0], [0, 0, 0], ("sphere", [0.065]))])
    w.link("upper_arm_link", (8.058, [-0.2125, 0, 0.138], cyl_inertia(8.058, 0.054, 0.425)),
           [([-0.2125, 0, 0.138], [0, h, 0], ("cylinder", [0.055, 0.34])),
            ([0, 0, 0.138], [0, 0, 0], ("sphere", [0.063])),
            ([-0.425, 0, 0.138], [0, 0, 0], ("sphere", [0.058]))])
    w.link("forearm_link", (2.846, [-0.2422, 0, 0.007], cyl_inertia(2.846, 0.04, 0.392)),
           [([-0.196, 0, 0.007], [0, h, 0], ("cylinder", [0.041, 0.32])),
            ([0, 0, 0.007], [0, 0, 0], ("sphere", [0.052])),
            ([-0.3922, 0, 0.02], [0, 0, 0], ("sphere", [0.046]))])
    w.link("wrist_1_link", (1.37, [0, -0.01, 0], cyl_inertia(1.37, 0.045, 0.1)),
           [([0, 0, 0], [0, 0, 0], ("cylinder", [0.046, 0.09])),
            ([0, -0.04, 0], [h, 0, 0], ("cylinder", [0.042, 0.05]))])
    w.link("wrist_2_link", (1.3, [0, 0.01, 0], cyl_inertia(1.3, 0.045, 0.1)),
           [([0, 0, 0], [0, 0, 0], ("cylinder", [0.046, 0.09])),
            ([0, 0.04, 0], [h, 0, 0], ("cylinder", [0.042, 0.05]))])
    w.link("wrist_3_link", (0.365, [0, 0, -0.02], cyl_inertia(0.365, 0.04, 0.04)),
           [([0, 0, -0.02], [0, 0, 0], ("cylinder", [0.04, 0.045])),
            ([0, 0, 0.01], [0, 0, 0], ("box", [0.06, 0.06, 0.02]))])
    w.link("tool0")
    lim = lambda lo, hi, v, e: (lo, hi, v, e)
    w.joint("base_joint", "fixed", "world", "base_link", [0, 0, 0], [0, 0, 0])
    w.joint("shoulder_pan_joint", "revolute", "base_link", "shoulder_link", [0, 0, 0.1625], [0, 0, 0], [0, 0, 1], lim(-2 * pi, 2 * pi, pi, 150))
    w.joint("shoulder_lift_joint", "revolute", "shoulder_link", "upper_arm_link", [0, 0, 0], [h, 0, 0], [0, 0, 1], lim(-2 * pi, 2 * pi, pi, 150))
    w.joint("elbow_joint", "revolute", "upper_arm_link", "forearm_link", [-0.425, 0, 0], [0, 0, 0], [0, 0, 1], lim(-pi, pi, pi, 150))
    w.joint("wrist_1_joint", "revolute", "forearm_link", "wrist_1_link", [-0.3922, 0, 0.1333], [0, 0, 0], [0, 0, 1], lim(-2 * pi, 2 * pi, pi, 28))
    w.joint("wrist_2_joint", "revolute", "wrist_1_link", "wrist_2_link", [0, -0.0997, 0], [h, 0, 0], [0, 0, 1], lim(-2 * pi, 2 * pi, pi, 28))
    w.joint("wrist_3_joint", "revolute", "wrist_2_link", "wrist_3_link", [0, 0.0996, 0], [h, pi, pi], [0, 0, 1], lim(-2 * pi, 2 * pi, pi, 28))
    w.joint("flange_joint", "fixed", "wrist_3_link", "tool0", [0, 0, 0], [0, 0, 0])
    with open(os.path.join(d, "ur5e.urdf"), "w") as fh:
        fh.write(w.text())
    write_srdf(os.path.join(d, "ur5e.srdf"), "ur5e", [
        ("base_link", "shoulder_link", "Adjacent"),
        ("shoulder_link", "upper_arm_link", "Adjacent"),
        ("upper_arm_link", "forearm_link", "Adjacent"),
        ("forearm_link", "wrist_1_link", "Adjacent"),
        ("wrist_1_link", "wrist_2_link", "Adjacent"),
        ("wrist_2_link", "wrist_3_link", "Adjacent"),
        ("wrist_1_link", "wrist_3_link", "Never"),
        ("base_link", "upper_arm_link", "Never"),
    ])


def gen_mobile(kind, links, joints, disabled):
    """Whole-body fixtures: world -x-> -y-> -yaw-> base_link; FR3 on top."""
    name = {"husky": "husky_fr3", "xls": "xls_fr3", "caster": "caster_fr3"}[kind]
    d = os.path.join(OUT, name)
    os.makedirs(d, exist_ok=True)
    w = UrdfWriter(name)
    big = 1e3
    w.link("world")
    w.link("virtual_x_link", (1e-3, [0, 0, 0], [1e-6, 0, 0, 1e-6, 0, 1e-6]))
    w.link("virtual_y_link", (1e-3, [0, 0, 0], [1e-6, 0, 0, 1e-6, 0, 1e-6]))
    if kind == "husky":
        # Husky A200-like chassis: 0.99 x 0.67 x 0.39 m, wheel r 0.165, track 0.555
        base_cols = [([0, 0, 0.22], [0, 0, 0], ("box", [0.98, 0.57, 0.24])),
                     ([0.3, 0, 0.40], [0, 0, 0], ("box", [0.30, 0.40, 0.12]))]
        w.link("base_link", (46.0, [0, 0, 0.2], [0.61, 0, 0, 1.3, 0, 1.6]), base_cols)
        wheels = [("wheel_left_joint", "wheel_left_link", [0, 0.2775, 0.165]),
                  ("wheel_right_joint", "wheel_right_link", [0, -0.2775, 0.165])]
        wheel_r, wheel_w = 0.165, 0.11
        mount = [0.25, 0, 0.34]
    elif kind == "caster":
        # two powered casters at (0.25, 0.2) and (-0.25, -0.2): steer axis z at the
        # position, wheel (r 0.08) trailing by the offset b = 0.05 along the steer
        # direction (the contact point of CasterFKJacobian, robot_data.cpp:193-196)
        base_cols = [([0, 0, 0.24], [0, 0, 0], ("box", [0.70, 0.52, 0.20]))]
        w.link("base_link", (40.0, [0, 0, 0.24], [0.9, 0, 0, 1.7, 0, 2.4]), base_cols)
        wheels = []
        for i, (px, py) in enumerate([(0.25, 0.2), (-0.25, -0.2)]):
            sl = "caster_%d_steer_link" % i
            w.link(sl, (0.8, [0, 0, 0], [1e-3, 0, 0, 1e-3, 0, 1e-3]))
            wheels.append(("wheel_c%d_0steer_joint" % i, sl, [px, py, 0.16], "steer"))
            wheels.append(("wheel_c%d_1drive_joint" % i, "caster_%d_wheel_link" % i, [0.05, 0, -0.08], sl))
        wheel_r, wheel_w = 0.08, 0.05
        mount = [0.15, 0, 0.34]
    else:
        # Summit-XLS-like chassis, mecanum wheels at (+-0.2225, +-0.2045), r 0.12
        base_cols = [([0, 0, 0.25], [0, 0, 0], ("box", [0.62, 0.30, 0.22]))]
        w.link("base_link", (60.0, [0, 0, 0.25], [1.1, 0, 0, 2.0, 0, 2.6]), base_cols)
        wheels = [("wheel_fl_joint", "wheel_fl_link", [0.2225, 0.2045, 0.12]),
                  ("wheel_fr_joint", "wheel_fr_link", [0.2225, -0.2045, 0.12]),
                  ("wheel_rl_joint", "wheel_rl_link", [-0.2225, 0.2045, 0.12]),
                  ("wheel_rr_joint", "wheel_rr_link", [-0.2225, -0.2045, 0.12])]
        wheel_r, wheel_w = 0.12, 0.09
        mount = [0.18, 0, 0.36]
    if kind == "caster":   # (joint, child, xyz, parent | "steer")
        wheels, casters = [(jn, wl, xyz) for (jn, wl, xyz, _) in wheels], wheels
    else:
        casters = None
    for (_, wl, _) in wheels:
        if casters and wl.endswith("steer_link"):
            continue
        w.link(wl, (2.6, [0, 0, 0], cyl_inertia(2.6, wheel_r, wheel_w)),
               [([0, 0, 0], [0, 0, 0], ("cylinder", [wheel_r, wheel_w]))])
    emit_fr3_arm(w, links, joints, mount_parent="base_link", mount_xyz=mount, skip_base=True)
    w.joint("virtual_0_x_joint", "prismatic", "world", "virtual_x_link", [0, 0, 0], [0, 0, 0], [1, 0, 0], (-big, big, 10.0, 1e4))
    w.joint("virtual_1_y_joint", "prismatic", "virtual_x_link", "virtual_y_link", [0, 0, 0], [0, 0, 0], [0, 1, 0], (-big, big, 10.0, 1e4))
    w.joint("virtual_2_yaw_joint", "revolute", "virtual_y_link", "base_link", [0, 0, 0], [0, 0, 0], [0, 0, 1], (-big, big, 10.0, 1e4))
    # wheel joints: declared revolute, wheel axis = link z, rotated so z is lateral
    if casters:   # steer: base_link -> steer link about z; drive: steer link -> wheel about the lateral axis
        for (jn, wl, xyz, par) in casters:
            if par == "steer":
                w.joint(jn, "revolute", "base_link", wl, xyz, [0, 0, 0], [0, 0, 1], (-big, big, 10.0, 100))
            else:
                w.joint(jn, "revolute", par, wl, xyz, [-math.pi / 2, 0, 0], [0, 0, 1], (-big, big, 30.0, 100))
        wheels = [(jn, wl, xyz) for (jn, wl, xyz, par) in casters if par != "steer"]
    else:
        for (jn, wl, xyz) in wheels:
            w.joint(jn, "revolute", "base_link", wl, xyz, [-math.pi / 2, 0, 0], [0, 0, 1], (-big, big, 30.0, 100))
    with open(os.path.join(d, name + ".urdf"), "w") as fh:
        fh.write(w.text())
    extra = [("base_link", "fr3_link0", "Adjacent"), ("base_link", "fr3_link1", "Never")]
    for (_, wl, _) in wheels:
        extra += [(wl, "base_link", "Adjacent"), (wl, "fr3_link0", "Never"), (wl, "fr3_link1", "Never")]
    for i, (_, a, _) in enumerate(wheels):
        for (_, b, _) in wheels[i + 1:]:
            extra.append((a, b, "Never"))
    write_srdf(os.path.join(d, name + ".srdf"), name, list(disabled) + extra)


def main():
    if not os.path.isdir(REF_FR3):
        sys.exit("reference FR3 model not found; fixtures are generated in the build container only")
    links, joints, disabled = read_reference_fr3()
    gen_fr3(links, joints, disabled)
    gen_ur5e()
    gen_mobile("husky", links, joints, disabled)
    gen_mobile("xls", links, joints, disabled)
    gen_mobile("caster", links, joints, disabled)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
