// URDF/SRDF subset reader and Pinocchio-convention model build.
//
// Restates (reference src/manipulator/robot_data.cpp:21-62):
//   pinocchio::urdf::buildModel    urdfdom orders a link's children by joint
//                                  name (std::map); Pinocchio walks the tree
//                                  depth first in that order; fixed joints
//                                  are merged into the moving parent.
//   pinocchio::urdf::buildGeom     COLLISION elements, file order per link,
//                                  placement = body placement * origin.
//   GeometryModel::addAllCollisionPairs   all (i<j) with different parent joints.
//   pinocchio::srdf::removeCollisionPairs drop pairs between disabled links.
//   lowerPositionLimit / velocityLimit    from <limit>.
#include "model.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>

#include "../../include/drc_amd.h"

namespace drc_amd {
namespace {

// ---------------------------------------------------------------- tiny XML
struct XmlNode {
  std::string tag;
  std::map<std::string, std::string> attr;
  std::vector<std::unique_ptr<XmlNode>> kids;
  const XmlNode* child(const char* t) const {
    for (auto& k : kids)
      if (k->tag == t) return k.get();
    return nullptr;
  }
  std::vector<const XmlNode*> children(const char* t) const {
    std::vector<const XmlNode*> r;
    for (auto& k : kids)
      if (k->tag == t) r.push_back(k.get());
    return r;
  }
  const char* get(const char* k, const char* def = nullptr) const {
    auto it = attr.find(k);
    return it == attr.end() ? def : it->second.c_str();
  }
};

class XmlParser {
 public:
  explicit XmlParser(const std::string& s) : s_(s) {}
  std::unique_ptr<XmlNode> parse(std::string* err) {
    std::unique_ptr<XmlNode> root;
    while (skip_misc()) {
      if (root) break;
      root = element(err);
      if (!root) return nullptr;
    }
    if (!root) *err = "no root element";
    return root;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  bool at(const char* p) const { return s_.compare(i_, std::strlen(p), p) == 0; }
  void ws() {
    while (i_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[i_]))) ++i_;
  }
  // skips whitespace, comments, <? ?> and <! > ; true if a '<' element follows
  bool skip_misc() {
    for (;;) {
      ws();
      if (i_ >= s_.size()) return false;
      if (at("<!--")) {
        size_t e = s_.find("-->", i_ + 4);
        i_ = e == std::string::npos ? s_.size() : e + 3;
      } else if (at("<?")) {
        size_t e = s_.find("?>", i_ + 2);
        i_ = e == std::string::npos ? s_.size() : e + 2;
      } else if (at("<!")) {
        size_t e = s_.find('>', i_ + 2);
        i_ = e == std::string::npos ? s_.size() : e + 1;
      } else if (s_[i_] == '<') {
        return true;
      } else {
        size_t e = s_.find('<', i_);  // text content: ignored
        i_ = e == std::string::npos ? s_.size() : e;
      }
    }
  }
  std::string name() {
    size_t b = i_;
    while (i_ < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[i_])) || s_[i_] == '_' ||
                              s_[i_] == ':' || s_[i_] == '-' || s_[i_] == '.'))
      ++i_;
    return s_.substr(b, i_ - b);
  }
  std::unique_ptr<XmlNode> element(std::string* err) {
    auto n = std::make_unique<XmlNode>();
    ++i_;  // '<'
    n->tag = name();
    if (n->tag.empty()) {
      *err = "malformed tag at byte " + std::to_string(i_);
      return nullptr;
    }
    for (;;) {
      ws();
      if (i_ >= s_.size()) {
        *err = "unterminated tag <" + n->tag + ">";
        return nullptr;
      }
      if (at("/>")) {
        i_ += 2;
        return n;
      }
      if (s_[i_] == '>') {
        ++i_;
        break;
      }
      std::string k = name();
      ws();
      if (k.empty() || i_ >= s_.size() || s_[i_] != '=') {
        *err = "malformed attribute in <" + n->tag + ">";
        return nullptr;
      }
      ++i_;
      ws();
      char q = s_[i_];
      if (q != '"' && q != '\'') {
        *err = "unquoted attribute in <" + n->tag + ">";
        return nullptr;
      }
      size_t e = s_.find(q, i_ + 1);
      if (e == std::string::npos) {
        *err = "unterminated attribute in <" + n->tag + ">";
        return nullptr;
      }
      n->attr[k] = s_.substr(i_ + 1, e - i_ - 1);
      i_ = e + 1;
    }
    for (;;) {
      if (!skip_misc()) {
        *err = "missing </" + n->tag + ">";
        return nullptr;
      }
      if (at("</")) {
        i_ += 2;
        std::string t = name();
        ws();
        if (t != n->tag || i_ >= s_.size() || s_[i_] != '>') {
          *err = "mismatched </" + t + "> for <" + n->tag + ">";
          return nullptr;
        }
        ++i_;
        return n;
      }
      auto k = element(err);
      if (!k) return nullptr;
      n->kids.push_back(std::move(k));
    }
  }
};

// ----------------------------------------------------------- SE(3) helpers
struct SE3 {
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  double p[3] = {0, 0, 0};
};
SE3 mul(const SE3& a, const SE3& b) {
  SE3 c;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      c.R[3 * i + j] = a.R[3 * i] * b.R[j] + a.R[3 * i + 1] * b.R[3 + j] + a.R[3 * i + 2] * b.R[6 + j];
    c.p[i] = a.R[3 * i] * b.p[0] + a.R[3 * i + 1] * b.p[1] + a.R[3 * i + 2] * b.p[2] + a.p[i];
  }
  return c;
}
bool parse_vec(const char* s, int n, double* out) {
  if (!s) return false;
  std::istringstream is(s);
  for (int i = 0; i < n; ++i)
    if (!(is >> out[i])) return false;
  return true;
}
// rpy -> Rz(y) Ry(p) Rx(r)
SE3 origin_of(const XmlNode* el) {
  SE3 T;
  const XmlNode* o = el ? el->child("origin") : nullptr;
  if (!o) return T;
  double xyz[3] = {0, 0, 0}, rpy[3] = {0, 0, 0};
  if (o->get("xyz")) parse_vec(o->get("xyz"), 3, xyz);
  if (o->get("rpy")) parse_vec(o->get("rpy"), 3, rpy);
  const double cr = std::cos(rpy[0]), sr = std::sin(rpy[0]), cp = std::cos(rpy[1]),
               sp = std::sin(rpy[1]), cy = std::cos(rpy[2]), sy = std::sin(rpy[2]);
  const double R[9] = {cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr,
                       sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr,
                       -sp,     cp * sr,                cp * cr};
  std::memcpy(T.R, R, sizeof(R));
  std::memcpy(T.p, xyz, sizeof(xyz));
  return T;
}
void put12(const SE3& T, double* out) {
  std::memcpy(out, T.R, 9 * sizeof(double));
  std::memcpy(out + 9, T.p, 3 * sizeof(double));
}
bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

struct Builder {
  const XmlNode* robot;
  std::map<std::string, const XmlNode*> links, joints;
  std::map<std::string, std::vector<std::string>> children;  // link -> joint names (sorted)
  HostModel* hm;
  std::vector<std::string> geom_link;
  std::map<std::string, int> frame_of_link;
  std::string err;

  bool add_link(const std::string& lname, int jid, const SE3& place) {
    DevModel& m = hm->dev;
    if (m.nframes >= kMaxFrames) return fail("too many links");
    frame_of_link[lname] = m.nframes;
    hm->frame_names.push_back(lname);
    m.frame_joint[m.nframes] = jid;
    put12(place, m.frame_place[m.nframes]);
    ++m.nframes;
    const XmlNode* ln = links[lname];
    int k = 0;
    for (const XmlNode* c : ln->children("collision")) {
      const XmlNode* g = c->child("geometry");
      if (!g || g->kids.empty()) return fail("collision without geometry in link " + lname);
      const XmlNode* s = g->kids[0].get();
      if (m.ngeom >= kMaxGeoms) return fail("too many collision geometries");
      int gi = m.ngeom;
      double prm[3] = {0, 0, 0};
      if (s->tag == "sphere") {
        m.gtype[gi] = kSphere;
        if (!parse_vec(s->get("radius"), 1, prm)) return fail("bad sphere radius");
        m.gbound[gi] = prm[0];
      } else if (s->tag == "cylinder") {
        m.gtype[gi] = kCylinder;
        double rl[2];
        if (!parse_vec(s->get("radius"), 1, rl) || !parse_vec(s->get("length"), 1, rl + 1))
          return fail("bad cylinder");
        prm[0] = rl[0];
        prm[1] = 0.5 * rl[1];
        m.gbound[gi] = rl[0];  // capsule core = axis segment
      } else if (s->tag == "box") {
        m.gtype[gi] = kBox;
        double sz[3];
        if (!parse_vec(s->get("size"), 3, sz)) return fail("bad box size");
        for (int i = 0; i < 3; ++i) prm[i] = 0.5 * sz[i];
        m.gbound[gi] = std::sqrt(prm[0] * prm[0] + prm[1] * prm[1] + prm[2] * prm[2]);
      } else {
        return fail("unsupported collision geometry <" + s->tag + "> (mesh) in link " + lname);
      }
      std::memcpy(m.gparam[gi], prm, sizeof(prm));
      m.gparent[gi] = jid;
      put12(mul(place, origin_of(c)), m.gplace[gi]);
      hm->geom_names.push_back(lname + "_" + std::to_string(k++));
      geom_link.push_back(lname);
      ++m.ngeom;
    }
    if (const XmlNode* ie = ln->child("inertial")) {
      // URDF <inertial>: mass, com origin, inertia about the com in the origin's
      // rotated frame; rotate into the joint frame and merge (parallel axis)
      const XmlNode* ms = ie->child("mass");
      const XmlNode* it = ie->child("inertia");
      double mass = 0;
      if (ms && ms->get("value") && !parse_vec(ms->get("value"), 1, &mass)) return fail("bad mass in link " + lname);
      double Il[6] = {0, 0, 0, 0, 0, 0};  // xx yy zz xy xz yz
      static const char* kI[6] = {"ixx", "iyy", "izz", "ixy", "ixz", "iyz"};
      for (int k2 = 0; k2 < 6; ++k2)
        if (it && it->get(kI[k2]) && !parse_vec(it->get(kI[k2]), 1, &Il[k2])) return fail("bad inertia in link " + lname);
      const SE3 T = mul(place, origin_of(ie));
      const double L[9] = {Il[0], Il[3], Il[4], Il[3], Il[1], Il[5], Il[4], Il[5], Il[2]};
      double RI[9], I[9];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) RI[3 * r + c] = T.R[3 * r] * L[c] + T.R[3 * r + 1] * L[3 + c] + T.R[3 * r + 2] * L[6 + c];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) I[3 * r + c] = RI[3 * r] * T.R[3 * c] + RI[3 * r + 1] * T.R[3 * c + 1] + RI[3 * r + 2] * T.R[3 * c + 2];
      double* b = m.inertia[jid];
      const double m0 = b[0], m1 = m0 + mass;
      double c0[3] = {b[1], b[2], b[3]}, c1[3];
      for (int i = 0; i < 3; ++i) c1[i] = m1 > 0 ? (m0 * c0[i] + mass * T.p[i]) / m1 : 0.0;
      // I_new(about c1) = I0 + m0 (|d0|^2 E - d0 d0^T) + I + mass (|d|^2 E - d d^T)
      double Inew[9];
      for (int i = 0; i < 9; ++i) Inew[i] = 0;
      const double I0[9] = {b[4], b[7], b[8], b[7], b[5], b[9], b[8], b[9], b[6]};
      auto add = [&](const double* Ib, double mb, const double* cb) {
        const double d[3] = {cb[0] - c1[0], cb[1] - c1[1], cb[2] - c1[2]};
        const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) Inew[3 * r + c] += Ib[3 * r + c] + mb * ((r == c ? dd : 0.0) - d[r] * d[c]);
      };
      add(I0, m0, c0);
      add(I, mass, T.p);
      b[0] = m1;
      for (int i = 0; i < 3; ++i) b[1 + i] = c1[i];
      b[4] = Inew[0]; b[5] = Inew[4]; b[6] = Inew[8];
      b[7] = Inew[1]; b[8] = Inew[2]; b[9] = Inew[5];
    }
    return true;
  }

  bool walk(const std::string& lname, int jid, const SE3& place) {
    if (!add_link(lname, jid, place)) return false;
    for (const std::string& jn : children[lname]) {
      const XmlNode* j = joints[jn];
      const std::string child = j->child("child")->get("link");
      SE3 jp = mul(place, origin_of(j));
      std::string type = j->get("type", "");
      if (type == "fixed") {
        if (!walk(child, jid, jp)) return false;
        continue;
      }
      if (type != "revolute" && type != "prismatic")
        return fail("unsupported joint type '" + type + "' (" + jn + "); continuous/floating/planar joints change nq (SURVEY H4b)");
      DevModel& m = hm->dev;
      if (m.nv >= kMaxJoints) return fail("too many joints");
      int id = ++m.nv;
      m.parent[id] = jid;
      m.jtype[id] = type == "revolute" ? kRevolute : kPrismatic;
      put12(jp, m.jplace[id]);
      double ax[3] = {1, 0, 0};
      if (const XmlNode* a = j->child("axis")) parse_vec(a->get("xyz"), 3, ax);
      double n = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
      for (int i = 0; i < 3; ++i) m.axis[id][i] = ax[i] / n;
      double lo = 0, hi = 0, vel = 0, eff = 0;
      if (const XmlNode* l = j->child("limit")) {
        if (l->get("lower")) parse_vec(l->get("lower"), 1, &lo);
        if (l->get("upper")) parse_vec(l->get("upper"), 1, &hi);
        if (l->get("velocity")) parse_vec(l->get("velocity"), 1, &vel);
        if (l->get("effort")) parse_vec(l->get("effort"), 1, &eff);
      }
      m.lower[id - 1] = lo;
      m.upper[id - 1] = hi;
      m.vel[id - 1] = vel;
      hm->effort.push_back(eff);
      hm->joint_names.push_back(jn);
      m.anc[id] = (jid > 0 ? m.anc[jid] : 0u) | (1u << (id - 1));
      if (!walk(child, id, SE3())) return false;
    }
    return true;
  }
  bool fail(const std::string& e) {
    err = e;
    return false;
  }
};

}  // namespace

int build_model_from_urdf(const std::string& urdf_path, const std::string& srdf_path,
                          HostModel* out, std::string* err) {
  std::string text;
  if (!read_file(urdf_path, &text)) {
    *err = "URDF file does not exist: " + urdf_path;
    return DRC_ERR_FILE;
  }
  XmlParser xp(text);
  auto root = xp.parse(err);
  if (!root) return DRC_ERR_PARSE;
  if (root->tag != "robot") {
    *err = "URDF root element is <" + root->tag + ">, expected <robot>";
    return DRC_ERR_PARSE;
  }
  *out = HostModel();
  Builder b;
  b.robot = root.get();
  b.hm = out;
  std::set<std::string> child_links;
  for (auto& k : root->kids) {
    if (k->tag == "link") b.links[k->get("name", "")] = k.get();
    if (k->tag == "joint") b.joints[k->get("name", "")] = k.get();
  }
  for (auto& kv : b.joints) {  // std::map: joint-name order, as urdfdom
    const XmlNode* p = kv.second->child("parent");
    const XmlNode* c = kv.second->child("child");
    if (!p || !c || !p->get("link") || !c->get("link")) {
      *err = "joint " + kv.first + " lacks parent/child";
      return DRC_ERR_PARSE;
    }
    if (!b.links.count(p->get("link")) || !b.links.count(c->get("link"))) {
      *err = "joint " + kv.first + " references an unknown link";
      return DRC_ERR_PARSE;
    }
    b.children[p->get("link")].push_back(kv.first);
    child_links.insert(c->get("link"));
  }
  std::vector<std::string> roots;
  for (auto& kv : b.links)
    if (!child_links.count(kv.first)) roots.push_back(kv.first);
  if (roots.size() != 1) {
    *err = "URDF must have exactly one root link";
    return DRC_ERR_PARSE;
  }
  if (!b.walk(roots[0], 0, SE3())) {
    *err = b.err;
    return DRC_ERR_UNSUPPORTED;
  }
  DevModel& m = out->dev;
  // addAllCollisionPairs
  std::vector<std::pair<int, int>> pairs;
  for (int i = 0; i < m.ngeom; ++i)
    for (int j = i + 1; j < m.ngeom; ++j)
      if (m.gparent[i] != m.gparent[j]) pairs.emplace_back(i, j);
  // srdf::removeCollisionPairs
  if (!srdf_path.empty()) {
    std::string st;
    if (read_file(srdf_path, &st)) {
      XmlParser sp(st);
      std::string e2;
      auto sr = sp.parse(&e2);
      if (!sr) {
        *err = "SRDF: " + e2;
        return DRC_ERR_PARSE;
      }
      std::set<std::pair<int, int>> drop;
      for (const XmlNode* d : sr->children("disable_collisions")) {
        const char* l1 = d->get("link1");
        const char* l2 = d->get("link2");
        if (!l1 || !l2 || !b.frame_of_link.count(l1) || !b.frame_of_link.count(l2)) continue;
        if (std::string(l1) == l2) continue;
        for (int a = 0; a < m.ngeom; ++a) {
          if (b.geom_link[a] != l1) continue;
          for (int c = 0; c < m.ngeom; ++c)
            if (b.geom_link[c] == l2) drop.insert({std::min(a, c), std::max(a, c)});
        }
      }
      std::vector<std::pair<int, int>> kept;
      for (auto& p : pairs)
        if (!drop.count(p)) kept.push_back(p);
      pairs.swap(kept);
    }
    // a missing SRDF keeps every pair (reference robot_data.cpp:44-48)
  }
  if (static_cast<int>(pairs.size()) > kMaxPairs) {
    *err = "too many collision pairs";
    return DRC_ERR_UNSUPPORTED;
  }
  m.npairs = static_cast<int>(pairs.size());
  for (int p = 0; p < m.npairs; ++p) {
    m.pair_a[p] = static_cast<int16_t>(pairs[p].first);
    m.pair_b[p] = static_cast<int16_t>(pairs[p].second);
  }
  // pair order of the wave kernel's closed-form / bound pass: by type class
  // (sphere-sphere, sphere-cylinder, sphere-box, cylinder-cylinder,
  // cylinder-box, box-box), pair index order within a class
  {
    int n = 0;
    for (int cls = 0; cls < 6; ++cls)
      for (int p = 0; p < m.npairs; ++p) {
        int ta = m.gtype[m.pair_a[p]], tb = m.gtype[m.pair_b[p]];
        if (ta > tb) std::swap(ta, tb);
        const int c = ta == 0 ? tb : (ta == 1 ? 2 + tb : 5);  // (0,0)0 (0,1)1 (0,2)2 (1,1)3 (1,2)4 (2,2)5
        if (c == cls) m.pair_order[n++] = static_cast<int16_t>(p);
      }
    for (int sl = 0; sl < m.npairs; ++sl) {
      m.slot_a[sl] = m.pair_a[m.pair_order[sl]];
      m.slot_b[sl] = m.pair_b[m.pair_order[sl]];
    }
  }
  // GJK candidate slots of the lane-per-instance task stage: the pairs with
  // no sphere (no closed form), numbered in pair order
  m.ncand_slots = 0;
  for (int p = 0; p < m.npairs; ++p) {
    m.cand_slot[p] = -1;
    if (m.gtype[m.pair_a[p]] != kSphere && m.gtype[m.pair_b[p]] != kSphere) {
      if (m.ncand_slots < kMaxCandSlots) m.cand_pair[m.ncand_slots] = static_cast<int16_t>(p);
      m.cand_slot[p] = static_cast<int16_t>(m.ncand_slots < kMaxCandSlots ? m.ncand_slots : -1);
      ++m.ncand_slots;
    }
  }
  return DRC_OK;
}

}  // namespace drc_amd
