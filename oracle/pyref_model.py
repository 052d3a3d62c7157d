"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

numpy restatement of the reference's model build:
``drc::Manipulator::RobotData::RobotData`` (src/manipulator/robot_data.cpp:7-70)
builds a Pinocchio model with ``pinocchio::urdf::buildModel`` (:21),
``buildGeom(COLLISION)`` (:27/:33), ``addAllCollisionPairs`` (:36) and
``srdf::removeCollisionPairs`` (:42).  Pinocchio/urdfdom are not available, so
their published conventions are restated here:

* urdfdom links children in joint-name (std::map) order; Pinocchio walks the
  tree depth-first in that order, so joint indices and geometry indices
  follow that traversal; collision elements of a link keep file order.
* fixed joints are merged: a link behind a fixed joint keeps the moving
  parent joint and a constant placement; its inertia is appended there.
* rpy → R = Rz(yaw) · Ry(pitch) · Rx(roll).
* addAllCollisionPairs: every (i<j) with different parent joints.
* removeCollisionPairs: drop (i,j) whose geometry parent *bodies* are a
  disabled (link1, link2) pair.
"""
import xml.etree.ElementTree as ET
import numpy as np

REVOLUTE, PRISMATIC = 0, 1
SPHERE, CYLINDER, BOX = 0, 1, 2


def rpy_to_R(r, p, y):
    cr, sr = np.cos(r), np.sin(r)
    cp, sp = np.cos(p), np.sin(p)
    cy, sy = np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def se3(R=None, p=None):
    T = np.eye(4)
    if R is not None:
        T[:3, :3] = R
    if p is not None:
        T[:3, 3] = p
    return T


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.eye(4)
    xyz = [float(x) for x in o.get("xyz", "0 0 0").split()]
    rpy = [float(x) for x in o.get("rpy", "0 0 0").split()]
    return se3(rpy_to_R(*rpy), xyz)


class Model:
    """Flat kinematic model in Pinocchio ordering (joint 0 = universe)."""

    def __init__(self):
        self.jname = ["universe"]
        self.jtype = [-1]
        self.jparent = [-1]
        self.jplacement = [np.eye(4)]
        self.jaxis = [np.zeros(3)]
        self.lower, self.upper, self.vel, self.effort = [], [], [], []
        self.frames = {}          # link name -> (parent joint, placement)
        self.geoms = []           # dict(name, parent_joint, link, placement, type, params)
        self.pairs = []
        # inertias per joint: list of (mass, com(3), I(3x3) about com, in joint frame)
        self.inertia = [[]]

    @property
    def nv(self):
        return len(self.jname) - 1

    def ancestors(self, j):
        """Joint ids (>=1) supporting joint j, root first, including j."""
        out = []
        while j > 0:
            out.append(j)
            j = self.jparent[j]
        return out[::-1]


def load_urdf(urdf_path, srdf_path=None):
    root = ET.parse(urdf_path).getroot()
    links = {ln.get("name"): ln for ln in root.findall("link")}
    joints = {j.get("name"): j for j in root.findall("joint")}
    children = {}
    child_links = set()
    for name in sorted(joints):                      # urdfdom: std::map order
        j = joints[name]
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        children.setdefault(p, []).append(name)
        child_links.add(c)
    roots = [ln for ln in links if ln not in child_links]
    assert len(roots) == 1, "URDF must have one root link"
    m = Model()

    def add_link_content(lname, jid, place):
        m.frames[lname] = (jid, place.copy())
        ln = links[lname]
        for k, c in enumerate(ln.findall("collision")):
            g = c.find("geometry")[0]
            if g.tag == "sphere":
                t, prm = SPHERE, [float(g.get("radius")), 0, 0]
            elif g.tag == "cylinder":
                t, prm = CYLINDER, [float(g.get("radius")), 0.5 * float(g.get("length")), 0]
            elif g.tag == "box":
                t, prm = BOX, [0.5 * float(x) for x in g.get("size").split()]
            else:
                raise ValueError("unsupported collision geometry " + g.tag)
            m.geoms.append(dict(name="%s_%d" % (lname, k), parent_joint=jid, link=lname,
                                placement=place @ _origin(c), type=t, params=np.array(prm)))
        ie = ln.find("inertial")
        if ie is not None:
            T = place @ _origin(ie)
            mass = float(ie.find("mass").get("value"))
            it = ie.find("inertia")
            g = lambda k: float(it.get(k, "0"))
            I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]])
            R = T[:3, :3]
            m.inertia[jid].append((mass, T[:3, 3].copy(), R @ I @ R.T))

    def walk(lname, jid, place):
        add_link_content(lname, jid, place)
        for jn in children.get(lname, []):
            j = joints[jn]
            child = j.find("child").get("link")
            jp = place @ _origin(j)
            jt = j.get("type")
            if jt == "fixed":
                walk(child, jid, jp)
                continue
            if jt not in ("revolute", "prismatic"):
                raise ValueError("unsupported joint type %s (SURVEY H4b)" % jt)
            ax = j.find("axis")
            axis = np.array([float(x) for x in ax.get("xyz").split()]) if ax is not None else np.array([1.0, 0, 0])
            axis = axis / np.linalg.norm(axis)
            lim = j.find("limit")
            m.jname.append(jn)
            m.jtype.append(REVOLUTE if jt == "revolute" else PRISMATIC)
            m.jparent.append(jid)
            m.jplacement.append(jp)
            m.jaxis.append(axis)
            m.lower.append(float(lim.get("lower", "0")) if lim is not None else 0.0)
            m.upper.append(float(lim.get("upper", "0")) if lim is not None else 0.0)
            m.vel.append(float(lim.get("velocity", "0")) if lim is not None else 0.0)
            m.effort.append(float(lim.get("effort", "0")) if lim is not None else 0.0)
            m.inertia.append([])
            walk(child, len(m.jname) - 1, np.eye(4))

    walk(roots[0], 0, np.eye(4))
    ng = len(m.geoms)
    for i in range(ng):
        for j in range(i + 1, ng):
            if m.geoms[i]["parent_joint"] != m.geoms[j]["parent_joint"]:
                m.pairs.append((i, j))
    if srdf_path:
        sr = ET.parse(srdf_path).getroot()
        for d in sr.findall("disable_collisions"):
            l1, l2 = d.get("link1"), d.get("link2")
            if l1 not in m.frames or l2 not in m.frames or l1 == l2:
                continue
            drop = set()
            for a, ga in enumerate(m.geoms):
                if ga["link"] != l1:
                    continue
                for b, gb in enumerate(m.geoms):
                    if gb["link"] != l2:
                        continue
                    drop.add((min(a, b), max(a, b)))
            m.pairs = [p for p in m.pairs if p not in drop]
    m.lower, m.upper, m.vel, m.effort = map(np.array, (m.lower, m.upper, m.vel, m.effort))
    return m
