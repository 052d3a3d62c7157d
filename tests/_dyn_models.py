"""Small synthetic URDFs for the dynamics known-answer tests (test infrastructure).

two_link(): planar 2R arm (joints about y, links along x) whose mass matrix,
gravity and Coriolis terms have the textbook closed forms (Spong, Robot
Modeling and Control, §7.4).  rank_deficient(): a 3R chain whose last link has
no <inertial>, so M(q) has a zero row/column and PinvCOD must return the
rank-2 pseudo-inverse (robot_data.cpp:118)."""
import os

import numpy as np

TWO_LINK = dict(m1=1.7, m2=0.9, l1=0.55, lc1=0.3, lc2=0.21, I1=0.031, I2=0.017)


def _inertial(m, com, iyy, ixx=None, izz=None):
    ixx = iyy if ixx is None else ixx
    izz = iyy if izz is None else izz
    return ('<inertial><origin xyz="%r %r %r" rpy="0 0 0"/><mass value="%r"/>'
            '<inertia ixx="%r" ixy="0" ixz="0" iyy="%r" iyz="0" izz="%r"/></inertial>'
            % (com[0], com[1], com[2], m, ixx, iyy, izz))


def two_link(dirpath):
    p = TWO_LINK
    urdf = f"""<?xml version="1.0"?>
<robot name="two_link">
  <link name="base"/>
  <link name="link1">{_inertial(p['m1'], (p['lc1'], 0, 0), p['I1'])}</link>
  <link name="link2">{_inertial(p['m2'], (p['lc2'], 0, 0), p['I2'])}</link>
  <joint name="j1" type="revolute"><parent link="base"/><child link="link1"/>
    <origin xyz="0 0 0" rpy="0 0 0"/><axis xyz="0 1 0"/><limit lower="-3" upper="3" velocity="2" effort="10"/></joint>
  <joint name="j2" type="revolute"><parent link="link1"/><child link="link2"/>
    <origin xyz="{p['l1']!r} 0 0" rpy="0 0 0"/><axis xyz="0 1 0"/><limit lower="-3" upper="3" velocity="2" effort="10"/></joint>
</robot>
"""
    path = os.path.join(dirpath, "two_link.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    return path


def two_link_closed_form(q, qd, grav=9.81):
    p = TWO_LINK
    m1, m2, l1, lc1, lc2, I1, I2 = (p[k] for k in ("m1", "m2", "l1", "lc1", "lc2", "I1", "I2"))
    c2, s2 = np.cos(q[1]), np.sin(q[1])
    M = np.array([[m1 * lc1 ** 2 + I1 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * c2) + I2,
                   m2 * (lc2 ** 2 + l1 * lc2 * c2) + I2],
                  [m2 * (lc2 ** 2 + l1 * lc2 * c2) + I2, m2 * lc2 ** 2 + I2]])
    # rotation about +y tilts +x towards -z: height of a point at distance r is -r sin(angle)
    g = np.array([-(m1 * lc1 + m2 * l1) * grav * np.cos(q[0]) - m2 * lc2 * grav * np.cos(q[0] + q[1]),
                  -m2 * lc2 * grav * np.cos(q[0] + q[1])])
    h = m2 * l1 * lc2 * s2
    c = np.array([-h * (2 * qd[0] * qd[1] + qd[1] ** 2), h * qd[0] ** 2])
    return M, g, c


def rank_deficient(dirpath):
    urdf = f"""<?xml version="1.0"?>
<robot name="rank_deficient">
  <link name="base"/>
  <link name="a">{_inertial(1.2, (0.1, 0.0, 0.05), 0.02, 0.01, 0.015)}</link>
  <link name="b">{_inertial(0.8, (0.0, 0.12, 0.0), 0.01, 0.012, 0.008)}</link>
  <link name="c"/>
  <joint name="j1" type="revolute"><parent link="base"/><child link="a"/>
    <origin xyz="0 0 0.1" rpy="0 0 0"/><axis xyz="0 0 1"/><limit lower="-3" upper="3" velocity="2" effort="10"/></joint>
  <joint name="j2" type="revolute"><parent link="a"/><child link="b"/>
    <origin xyz="0.2 0 0" rpy="0 0.3 0"/><axis xyz="1 0 0"/><limit lower="-3" upper="3" velocity="2" effort="10"/></joint>
  <joint name="j3" type="revolute"><parent link="b"/><child link="c"/>
    <origin xyz="0 0.25 0" rpy="0 0 0"/><axis xyz="0 0 1"/><limit lower="-3" upper="3" velocity="2" effort="10"/></joint>
</robot>
"""
    path = os.path.join(dirpath, "rank_deficient.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    return path
