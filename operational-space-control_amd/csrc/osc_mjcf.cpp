// osc_mjcf.cpp -- MJCF (MuJoCo XML) reader for the kinematics front end (include/osc_kinematics.h:
// osc_kin_desc_from_mjcf / osc_kin_desc_from_mjcf_robot).
//
// The reference's controller is constructed from the robot's MJCF path and resolves its task
// sites and bodies by name when it loads it (unitree_go2/operational_space_controller.h:108-152,
// mj_loadXML + mj_name2id).  MuJoCo is not linked here, so this file restates the part of
// MuJoCo 3.2.7's compiler that update_osc_data's outputs depend on: the body tree (frames,
// joints, inertias, armature), the sites, gravity, and the default-class / childclass
// inheritance those attributes are usually written with.  Everything else (geoms, actuators,
// sensors, contact, assets, visuals) is parsed and skipped.
//
// Host-only C++17; no XML library (a small non-validating parser below).
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "osc_batch.h"
#include "osc_kinematics.h"

// osc_model.cpp: the body / site lists of a robot's YAML config (same file osc_desc_from_yaml
// reads), and the default config path.
int osc_config_lists(const char* robot, const char* yaml_path, std::vector<std::string>* bodies,
                     std::vector<std::string>* sites);

namespace {

// ------------------------------------------------------------------ minimal XML DOM
struct XNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attr;
  std::vector<std::unique_ptr<XNode>> kids;
  XNode* parent = nullptr;
  const std::string* get(const char* k) const {
    for (const auto& a : attr)
      if (a.first == k) return &a.second;
    return nullptr;
  }
};

class XmlParser {
 public:
  explicit XmlParser(const std::string& s) : s_(s) {}
  std::unique_ptr<XNode> parse(std::string* err) {
    auto root = std::make_unique<XNode>();
    root->tag = "#document";
    XNode* cur = root.get();
    while (p_ < s_.size()) {
      if (s_[p_] != '<') {   // character data: ignored (MJCF carries everything in attributes)
        ++p_;
        continue;
      }
      if (starts("<!--")) {
        const size_t e = s_.find("-->", p_ + 4);
        if (e == std::string::npos) return fail(err, "unterminated comment");
        p_ = e + 3;
      } else if (starts("<?")) {
        const size_t e = s_.find("?>", p_ + 2);
        if (e == std::string::npos) return fail(err, "unterminated declaration");
        p_ = e + 2;
      } else if (starts("<!")) {
        const size_t e = s_.find('>', p_ + 2);
        if (e == std::string::npos) return fail(err, "unterminated <!");
        p_ = e + 1;
      } else if (starts("</")) {
        p_ += 2;
        const std::string name = ident();
        skip_ws();
        if (p_ >= s_.size() || s_[p_] != '>') return fail(err, "bad closing tag");
        ++p_;
        if (cur == root.get() || cur->tag != name) return fail(err, "mismatched </" + name + ">");
        cur = cur->parent;
      } else {
        ++p_;
        auto node = std::make_unique<XNode>();
        node->tag = ident();
        if (node->tag.empty()) return fail(err, "empty tag name");
        bool closed = false;
        for (;;) {
          skip_ws();
          if (p_ >= s_.size()) return fail(err, "unterminated tag <" + node->tag + ">");
          if (s_[p_] == '/') {
            if (p_ + 1 >= s_.size() || s_[p_ + 1] != '>') return fail(err, "bad '/'");
            p_ += 2;
            closed = true;
            break;
          }
          if (s_[p_] == '>') {
            ++p_;
            break;
          }
          std::string k = ident();
          if (k.empty()) return fail(err, "bad attribute in <" + node->tag + ">");
          skip_ws();
          if (p_ >= s_.size() || s_[p_] != '=') return fail(err, "attribute without value");
          ++p_;
          skip_ws();
          if (p_ >= s_.size() || (s_[p_] != '"' && s_[p_] != '\'')) return fail(err, "unquoted value");
          const char q = s_[p_++];
          const size_t e = s_.find(q, p_);
          if (e == std::string::npos) return fail(err, "unterminated value");
          node->attr.emplace_back(k, unescape(s_.substr(p_, e - p_)));
          p_ = e + 1;
        }
        node->parent = cur;
        XNode* raw = node.get();
        cur->kids.push_back(std::move(node));
        if (!closed) cur = raw;
      }
    }
    if (cur != root.get()) return fail(err, "unclosed <" + cur->tag + ">");
    return root;
  }

 private:
  bool starts(const char* t) const { return s_.compare(p_, std::strlen(t), t) == 0; }
  void skip_ws() {
    while (p_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[p_]))) ++p_;
  }
  std::string ident() {
    const size_t a = p_;
    while (p_ < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[p_])) || s_[p_] == '_' ||
                              s_[p_] == '-' || s_[p_] == ':' || s_[p_] == '.'))
      ++p_;
    return s_.substr(a, p_ - a);
  }
  static std::string unescape(const std::string& v) {
    if (v.find('&') == std::string::npos) return v;
    static const std::pair<const char*, char> ents[] = {
        {"&lt;", '<'}, {"&gt;", '>'}, {"&amp;", '&'}, {"&quot;", '"'}, {"&apos;", '\''}};
    std::string o;
    for (size_t i = 0; i < v.size();) {
      bool hit = false;
      for (const auto& e : ents) {
        const size_t n = std::strlen(e.first);
        if (v.compare(i, n, e.first) == 0) {
          o.push_back(e.second);
          i += n;
          hit = true;
          break;
        }
      }
      if (!hit) o.push_back(v[i++]);
    }
    return o;
  }
  std::unique_ptr<XNode> fail(std::string* err, const std::string& m) {
    if (err) *err = m;
    return nullptr;
  }
  const std::string& s_;
  size_t p_ = 0;
};

// <include file="..."/>: the included file's <mujoco> children replace the element, wherever it
// sits (MuJoCo's xml_util include expansion); file names are relative to the main model file's
// directory.  Nested includes are expanded too (depth-limited, so a cycle is an error).
bool read_text(const std::string& path, std::string* out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  std::stringstream ss;
  ss << in.rdbuf();
  *out = ss.str();
  return true;
}

bool expand_includes(XNode* node, const std::string& dir, int depth, std::string* err) {
  std::vector<std::unique_ptr<XNode>> kids;
  for (auto& kp : node->kids) {
    if (kp->tag != "include") {
      if (!expand_includes(kp.get(), dir, depth, err)) return false;
      kids.push_back(std::move(kp));
      continue;
    }
    const std::string* f = kp->get("file");
    if (!f || f->empty()) {
      *err = "<include> without file";
      return false;
    }
    if (depth >= 16) {
      *err = "<include> nesting too deep (cycle?) at " + *f;
      return false;
    }
    const std::string path = (!f->empty() && (*f)[0] == '/') ? *f : dir + "/" + *f;
    std::string text;
    if (!read_text(path, &text)) {
      *err = "cannot open included file " + path;
      return false;
    }
    std::string perr;
    XmlParser parser(text);
    std::unique_ptr<XNode> root = parser.parse(&perr);
    if (!root) {
      *err = path + ": " + perr;
      return false;
    }
    XNode* mj = nullptr;
    for (auto& k : root->kids)
      if (k->tag == "mujoco") mj = k.get();
    if (!mj) {
      *err = path + ": included file has no <mujoco> element";
      return false;
    }
    if (!expand_includes(mj, dir, depth + 1, err)) return false;
    for (auto& k : mj->kids) {
      k->parent = node;
      kids.push_back(std::move(k));
    }
  }
  node->kids.swap(kids);
  return true;
}

// ------------------------------------------------------------------ small math
struct Quat {
  double w = 1, x = 0, y = 0, z = 0;
};
Quat qmul(const Quat& a, const Quat& b) {
  return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
          a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
Quat qnorm(Quat q) {
  const double n = std::sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  if (!(n > 0)) return Quat{};
  q.w /= n; q.x /= n; q.y /= n; q.z /= n;
  return q;
}
Quat axis_angle(const double* a, double ang) {
  const double n = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  if (!(n > 0)) return Quat{};
  const double s = std::sin(ang / 2) / n;
  return qnorm({std::cos(ang / 2), a[0] * s, a[1] * s, a[2] * s});
}
// rotation matrix (row-major, columns = frame axes) -> quaternion
Quat mat2quat(const double* R) {
  Quat q;
  const double tr = R[0] + R[4] + R[8];
  if (tr > 0) {
    const double s = std::sqrt(tr + 1.0) * 2;
    q = {0.25 * s, (R[7] - R[5]) / s, (R[2] - R[6]) / s, (R[3] - R[1]) / s};
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2;
    q = {(R[7] - R[5]) / s, 0.25 * s, (R[1] + R[3]) / s, (R[2] + R[6]) / s};
  } else if (R[4] > R[8]) {
    const double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2;
    q = {(R[2] - R[6]) / s, (R[1] + R[3]) / s, 0.25 * s, (R[5] + R[7]) / s};
  } else {
    const double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2;
    q = {(R[3] - R[1]) / s, (R[2] + R[6]) / s, (R[5] + R[7]) / s, 0.25 * s};
  }
  if (q.w < 0) q = {-q.w, -q.x, -q.y, -q.z};
  return qnorm(q);
}
// symmetric 3x3 eigen-decomposition (cyclic Jacobi); columns of V = eigenvectors
void eig3(const double* A, double* lam, double* V) {
  double a[9];
  std::memcpy(a, A, sizeof(a));
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    const double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    if (off < 1e-30 * (a[0] * a[0] + a[4] * a[4] + a[8] * a[8]) || off == 0.0) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        const double apq = a[3 * p + q];
        if (apq == 0.0) continue;
        const double th = 0.5 * (a[3 * q + q] - a[3 * p + p]) / apq;
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {   // A <- A G
          const double akp = a[3 * k + p], akq = a[3 * k + q];
          a[3 * k + p] = c * akp - s * akq;
          a[3 * k + q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {   // A <- G' A
          const double apk = a[3 * p + k], aqk = a[3 * q + k];
          a[3 * p + k] = c * apk - s * aqk;
          a[3 * q + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {   // V <- V G
          const double vkp = V[3 * k + p], vkq = V[3 * k + q];
          V[3 * k + p] = c * vkp - s * vkq;
          V[3 * k + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < 3; ++i) lam[i] = a[4 * i];
}

bool nums(const std::string* s, double* out, int n) {
  if (!s) return false;
  std::istringstream in(*s);
  for (int i = 0; i < n; ++i)
    if (!(in >> out[i])) return false;
  std::string rest;
  return !(in >> rest);
}

// ------------------------------------------------------------------ the compiler subset
struct Compiler {
  bool degree = true;            // MuJoCo's default angle unit
  std::string eulerseq = "xyz";
  int inertiafromgeom = 2;       // 0 false, 1 true, 2 auto (MuJoCo's default)
  int group_lo = 0, group_hi = 5;   // inertiagrouprange
};

struct DefaultClass {
  std::map<std::string, std::map<std::string, std::string>> elem;   // tag -> attr -> value
  const DefaultClass* parent = nullptr;
  const std::string* lookup(const std::string& tag, const char* key) const {
    for (const DefaultClass* c = this; c; c = c->parent) {
      auto t = c->elem.find(tag);
      if (t == c->elem.end()) continue;
      auto a = t->second.find(key);
      if (a != t->second.end()) return &a->second;
    }
    return nullptr;
  }
};

constexpr int kMaxRaw = 64;   // bodies as written, before welded bodies are fused

// osc_kin_desc's body fields with room for the bodies as written in the file
struct RawDesc {
  int nbody = 0;
  double gravity[3] = {0.0, 0.0, -9.81};
  int parent[kMaxRaw];
  int jnt_type[kMaxRaw];
  double pos[kMaxRaw][3], quat[kMaxRaw][4], axis[kMaxRaw][3], jnt_pos[kMaxRaw][3];
  double armature[kMaxRaw], mass[kMaxRaw], ipos[kMaxRaw][3], iquat[kMaxRaw][4], inertia[kMaxRaw][3];
};

void quat2mat(const double* q, double* R) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  const double n = std::sqrt(w * w + x * x + y * y + z * z);
  w /= n; x /= n; y /= n; z /= n;
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}

// one <joint> / <freejoint> as written (its class defaults resolved)
struct JointSpec {
  int type = OSC_KIN_JOINT_HINGE;
  double axis[3] = {0.0, 0.0, 1.0};
  double pos[3] = {0.0, 0.0, 0.0};
  double armature = 0.0;
};

// mass, COM and inertia about the COM (body frame) of one geom or a sum of them
struct MassProps {
  double m = 0.0, c[3] = {0.0, 0.0, 0.0}, I[9] = {0.0};
};

// a += b: combined mass, COM and inertia about the combined COM (parallel-axis theorem)
void mass_add(MassProps* a, const MassProps& b) {
  const double m = a->m + b.m;
  if (!(m > 0.0)) return;
  double c[3];
  for (int i = 0; i < 3; ++i) c[i] = (a->m * a->c[i] + b.m * b.c[i]) / m;
  double I[9];
  for (int k = 0; k < 9; ++k) I[k] = a->I[k] + b.I[k];
  const MassProps* parts[2] = {a, &b};
  for (const MassProps* q : parts) {
    const double dv[3] = {q->c[0] - c[0], q->c[1] - c[1], q->c[2] - c[2]};
    const double dd = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) I[3 * i + j] += q->m * ((i == j ? dd : 0.0) - dv[i] * dv[j]);
  }
  a->m = m;
  for (int i = 0; i < 3; ++i) a->c[i] = c[i];
  for (int k = 0; k < 9; ++k) a->I[k] = I[k];
}

struct Loader {
  Compiler comp;
  std::map<std::string, std::unique_ptr<DefaultClass>> classes;
  std::string err;
  RawDesc* d = nullptr;
  std::vector<std::string> body_name;        // per desc body
  struct Site {
    std::string name;
    int body;                                // desc index, -1 = world
    double pos[3];
  };
  std::vector<Site> sites;                   // model order

  bool fail(const std::string& m) {
    if (err.empty()) err = m;
    return false;
  }

  bool read_defaults(const XNode& n, const DefaultClass* parent) {
    const std::string* cname = n.get("class");
    std::string name = cname ? *cname : "main";
    if (!parent && cname && *cname != "main") return fail("top-level <default> must be class main");
    auto cls = std::make_unique<DefaultClass>();
    cls->parent = parent;
    DefaultClass* raw = cls.get();
    if (classes.count(name)) return fail("duplicate default class " + name);
    classes[name] = std::move(cls);
    for (const auto& k : n.kids) {
      if (k->tag == "default") {
        if (!read_defaults(*k, raw)) return false;
      } else {
        auto& m = raw->elem[k->tag];
        for (const auto& a : k->attr) m[a.first] = a.second;
      }
    }
    return true;
  }

  const DefaultClass* cls_of(const XNode& e, const DefaultClass* active) {
    if (const std::string* c = e.get("class")) {
      auto it = classes.find(*c);
      if (it == classes.end()) {
        fail("unknown default class " + *c);
        return nullptr;
      }
      return it->second.get();
    }
    return active;
  }
  // attribute of element e: its own, else its class chain
  const std::string* attr(const XNode& e, const DefaultClass* cls, const char* key) {
    if (const std::string* v = e.get(key)) return v;
    return cls ? cls->lookup(e.tag == "freejoint" ? "joint" : e.tag, key) : nullptr;
  }

  double angle(double a) const { return comp.degree ? a * M_PI / 180.0 : a; }

  // MuJoCo's frame orientation alternatives (quat | axisangle | euler | xyaxes | zaxis)
  bool orientation(const XNode& e, const DefaultClass* cls, Quat* q) {
    double v[6];
    int given = 0;
    Quat r;
    if (const std::string* s = attr(e, cls, "quat")) {
      if (!nums(s, v, 4)) return fail("bad quat in <" + e.tag + ">");
      r = qnorm({v[0], v[1], v[2], v[3]});
      ++given;
    }
    if (const std::string* s = attr(e, cls, "axisangle")) {
      if (!nums(s, v, 4)) return fail("bad axisangle");
      r = axis_angle(v, angle(v[3]));
      ++given;
    }
    if (const std::string* s = attr(e, cls, "euler")) {
      if (!nums(s, v, 3)) return fail("bad euler");
      if (comp.eulerseq.size() != 3) return fail("bad eulerseq");
      Quat acc;
      for (int i = 0; i < 3; ++i) {
        const char c = comp.eulerseq[i];
        double ax[3] = {0, 0, 0};
        const char lc = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
        if (lc < 'x' || lc > 'z') return fail("bad eulerseq");
        ax[lc - 'x'] = 1.0;
        const Quat t = axis_angle(ax, angle(v[i]));
        acc = (c == lc) ? qmul(acc, t) : qmul(t, acc);   // lower case: intrinsic (moving axes)
      }
      r = qnorm(acc);
      ++given;
    }
    if (const std::string* s = attr(e, cls, "xyaxes")) {
      if (!nums(s, v, 6)) return fail("bad xyaxes");
      double x[3] = {v[0], v[1], v[2]}, y[3] = {v[3], v[4], v[5]};
      const double nx = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      for (double& t : x) t /= nx;
      const double dp = x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
      for (int i = 0; i < 3; ++i) y[i] -= dp * x[i];
      const double ny = std::sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
      for (double& t : y) t /= ny;
      const double z[3] = {x[1] * y[2] - x[2] * y[1], x[2] * y[0] - x[0] * y[2], x[0] * y[1] - x[1] * y[0]};
      const double R[9] = {x[0], y[0], z[0], x[1], y[1], z[1], x[2], y[2], z[2]};
      r = mat2quat(R);
      ++given;
    }
    if (const std::string* s = attr(e, cls, "zaxis")) {
      if (!nums(s, v, 3)) return fail("bad zaxis");
      const double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      const double z[3] = {v[0] / n, v[1] / n, v[2] / n};
      // minimal rotation taking (0, 0, 1) to z
      const double ax[3] = {-z[1], z[0], 0.0};
      const double s2 = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1]);
      if (s2 < 1e-14) {
        r = z[2] > 0 ? Quat{} : Quat{0, 1, 0, 0};
      } else {
        r = axis_angle(ax, std::atan2(s2, z[2]));
      }
      ++given;
    }
    if (given > 1) return fail("more than one orientation in <" + e.tag + ">");
    *q = r;
    return true;
  }

  int new_body(int parent, const std::string& name) {
    const int b = d->nbody;
    if (b >= kMaxRaw) {
      fail("too many bodies");
      return -1;
    }
    ++d->nbody;
    body_name.push_back(name);
    d->parent[b] = parent;
    d->jnt_type[b] = OSC_KIN_JOINT_NONE;
    d->quat[b][0] = 1.0;
    d->iquat[b][0] = 1.0;
    d->axis[b][2] = 1.0;
    return b;
  }

  bool joint(const XNode& k, const DefaultClass* active, JointSpec* j) {
    const DefaultClass* c = cls_of(k, active);
    if (!err.empty()) return false;
    std::string type = k.tag == "freejoint" ? "free" : "hinge";
    if (k.tag == "joint")
      if (const std::string* t = attr(k, c, "type")) type = *t;
    if (type == "free") j->type = OSC_KIN_JOINT_FREE;
    else if (type == "ball") j->type = OSC_KIN_JOINT_BALL;
    else if (type == "slide") j->type = OSC_KIN_JOINT_SLIDE;
    else if (type == "hinge") j->type = OSC_KIN_JOINT_HINGE;
    else return fail("unsupported joint type " + type);
    if (j->type == OSC_KIN_JOINT_HINGE || j->type == OSC_KIN_JOINT_SLIDE)
      if (const std::string* a = attr(k, c, "axis"))
        if (!nums(a, j->axis, 3)) return fail("bad joint axis");
    if (j->type != OSC_KIN_JOINT_FREE)
      if (const std::string* p = attr(k, c, "pos"))
        if (!nums(p, j->pos, 3)) return fail("bad joint pos");
    if (const std::string* a = attr(k, c, "armature"))
      if (!nums(a, &j->armature, 1)) return fail("bad armature");
    // ref shifts qpos0 (the pose is computed at q - ref): not modelled, so refused
    if (const std::string* r = attr(k, c, "ref")) {
      double v = 0.0;
      if (!nums(r, &v, 1)) return fail("bad joint ref");
      if (v != 0.0) return fail("joint ref != 0 unsupported (qpos0 offset)");
    }
    return true;
  }

  // MuJoCo's geom mass properties (mjCGeom: density 1000 unless mass is given, principal
  // inertia of the primitive about its centre, placed by pos / orientation | fromto).
  // `used` = false for geoms outside inertiagrouprange (ignored, as MuJoCo does).
  bool geom_mass(const XNode& g, const DefaultClass* active, MassProps* out, bool* used) {
    const DefaultClass* c = cls_of(g, active);
    if (!err.empty()) return false;
    *used = false;
    double grp = 0.0;
    if (const std::string* s = attr(g, c, "group"))
      if (!nums(s, &grp, 1)) return fail("bad geom group");
    if (grp < comp.group_lo || grp > comp.group_hi) return true;
    *used = true;
    std::string type = "sphere";
    if (const std::string* t = attr(g, c, "type")) type = *t;
    if (type == "mesh" || type == "sdf" || type == "hfield")
      return fail("inertia from " + type + " geoms unsupported (give the body an <inertial>)");
    if (type == "plane") return fail("plane geom in a moving body");
    double size[3] = {0.0, 0.0, 0.0};
    if (const std::string* sz = attr(g, c, "size")) {
      std::istringstream in(*sz);
      int n = 0;
      while (n < 3 && (in >> size[n])) ++n;
    }
    double pos[3] = {0.0, 0.0, 0.0};
    Quat q;
    if (const std::string* ft = attr(g, c, "fromto")) {
      if (type != "capsule" && type != "cylinder" && type != "box" && type != "ellipsoid")
        return fail("fromto on a " + type + " geom");
      double v[6];
      if (!nums(ft, v, 6)) return fail("bad geom fromto");
      const double dz[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
      const double len = std::sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2]);
      if (!(len > 0.0)) return fail("degenerate geom fromto");
      for (int i = 0; i < 3; ++i) pos[i] = 0.5 * (v[i] + v[3 + i]);
      // half-length along the geom's z: size[1] (capsule, cylinder) or size[2] (box, ellipsoid)
      size[(type == "capsule" || type == "cylinder") ? 1 : 2] = 0.5 * len;
      const double z[3] = {dz[0] / len, dz[1] / len, dz[2] / len};
      const double ax[3] = {-z[1], z[0], 0.0};
      const double s2 = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1]);
      q = s2 < 1e-14 ? (z[2] > 0 ? Quat{} : Quat{0, 1, 0, 0}) : axis_angle(ax, std::atan2(s2, z[2]));
    } else {
      if (const std::string* p = attr(g, c, "pos"))
        if (!nums(p, pos, 3)) return fail("bad geom pos");
      if (!orientation(g, c, &q)) return false;
    }
    double vol = 0.0, Id[3] = {0.0, 0.0, 0.0};   // volume; principal inertia per unit mass
    const double r = size[0];
    if (type == "sphere") {
      vol = 4.0 / 3.0 * M_PI * r * r * r;
      Id[0] = Id[1] = Id[2] = 0.4 * r * r;
    } else if (type == "capsule" || type == "cylinder") {
      const double h = size[1], H = 2.0 * h;
      const double vc = M_PI * r * r * H;
      if (type == "cylinder") {
        vol = vc;
        Id[0] = Id[1] = (3.0 * r * r + H * H) / 12.0;
        Id[2] = 0.5 * r * r;
      } else {   // cylinder + two hemispheres (each's COM 3r/8 off its flat face)
        const double vs = 4.0 / 3.0 * M_PI * r * r * r;
        vol = vc + vs;
        const double Ixc = vc * (3.0 * r * r + H * H) / 12.0;
        const double Ixs = vs * (0.4 * r * r + h * h + 0.75 * h * r);
        Id[0] = Id[1] = (Ixc + Ixs) / vol;
        Id[2] = (vc * 0.5 * r * r + vs * 0.4 * r * r) / vol;
      }
    } else if (type == "box") {
      vol = 8.0 * size[0] * size[1] * size[2];
      Id[0] = (size[1] * size[1] + size[2] * size[2]) / 3.0;
      Id[1] = (size[0] * size[0] + size[2] * size[2]) / 3.0;
      Id[2] = (size[0] * size[0] + size[1] * size[1]) / 3.0;
    } else if (type == "ellipsoid") {
      vol = 4.0 / 3.0 * M_PI * size[0] * size[1] * size[2];
      Id[0] = (size[1] * size[1] + size[2] * size[2]) / 5.0;
      Id[1] = (size[0] * size[0] + size[2] * size[2]) / 5.0;
      Id[2] = (size[0] * size[0] + size[1] * size[1]) / 5.0;
    } else {
      return fail("unsupported geom type " + type);
    }
    double mass = 0.0;
    if (const std::string* ms = attr(g, c, "mass")) {
      if (!nums(ms, &mass, 1) || mass < 0.0) return fail("bad geom mass");
    } else {
      double rho = 1000.0;
      if (const std::string* dn = attr(g, c, "density"))
        if (!nums(dn, &rho, 1) || rho < 0.0) return fail("bad geom density");
      mass = rho * vol;
    }
    if (mass > 0.0 && !(vol > 0.0)) return fail("geom with mass but no volume");
    if (const std::string* sh = attr(g, c, "shellinertia"))
      if (*sh == "true") return fail("shellinertia unsupported");
    double R[9];
    const double qa[4] = {q.w, q.x, q.y, q.z};
    quat2mat(qa, R);
    out->m = mass;
    for (int i = 0; i < 3; ++i) out->c[i] = pos[i];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double t = 0.0;
        for (int k = 0; k < 3; ++k) t += R[3 * i + k] * Id[k] * R[3 * j + k];
        out->I[3 * i + j] = mass * t;
      }
    return true;
  }

  // principal frame of a body-frame inertia tensor -> ipos / iquat / inertia of body b
  void set_inertia(int b, const MassProps& mp) {
    double lam[3], V[9];
    eig3(mp.I, lam, V);
    const double det = V[0] * (V[4] * V[8] - V[5] * V[7]) - V[1] * (V[3] * V[8] - V[5] * V[6]) +
                       V[2] * (V[3] * V[7] - V[4] * V[6]);
    if (det < 0)
      for (int i = 0; i < 3; ++i) V[3 * i + 2] = -V[3 * i + 2];
    const Quat iq = mat2quat(V);
    d->mass[b] = mp.m;
    for (int i = 0; i < 3; ++i) {
      d->ipos[b][i] = mp.c[i];
      d->inertia[b][i] = lam[i] < 0.0 ? 0.0 : lam[i];
    }
    d->iquat[b][0] = iq.w; d->iquat[b][1] = iq.x; d->iquat[b][2] = iq.y; d->iquat[b][3] = iq.z;
  }

  // A body with k > 1 joints becomes a chain of k bodies, one joint each, exactly as
  // mj_kinematics composes a body's joints in order: the first carries the body's frame
  // (pos, orientation), the others sit at zero offset in the frame the previous joint left,
  // and the last (the body proper: its name, inertia, sites, children) gets everything else.
  // The leading chain bodies are massless.
  bool body(const XNode& n, int parent, const DefaultClass* active) {
    const std::string* nm = n.get("name");
    const std::string name = nm ? *nm : "";
    if (const std::string* cc = n.get("childclass")) {
      auto it = classes.find(*cc);
      if (it == classes.end()) return fail("unknown childclass " + *cc);
      active = it->second.get();
    }
    std::vector<JointSpec> js;
    for (const auto& kp : n.kids)
      if (kp->tag == "joint" || kp->tag == "freejoint") {
        js.emplace_back();
        if (!joint(*kp, active, &js.back())) return false;
      }
    for (size_t i = 0; i < js.size(); ++i) {
      if (js[i].type == OSC_KIN_JOINT_FREE && (js.size() > 1 || parent >= 0))
        return fail("free joint must be the only joint of a top-level body (" + name + ")");
      // MuJoCo's ball dofs turn about the body's FINAL axes (mj_comPos); they are the ball's own
      // only when no rotating joint follows it on the body
      if (js[i].type == OSC_KIN_JOINT_BALL)
        for (size_t k = i + 1; k < js.size(); ++k)
          if (js[k].type == OSC_KIN_JOINT_BALL || js[k].type == OSC_KIN_JOINT_HINGE)
            return fail("ball joint followed by a rotating joint on body " + name);
    }
    int b = new_body(parent, js.size() > 1 ? "" : name);
    if (b < 0) return false;
    if (n.get("pos") && !nums(n.get("pos"), d->pos[b], 3)) return fail("bad body pos");
    Quat q;
    if (!orientation(n, nullptr, &q)) return false;
    d->quat[b][0] = q.w; d->quat[b][1] = q.x; d->quat[b][2] = q.y; d->quat[b][3] = q.z;
    for (size_t i = 0; i < js.size(); ++i) {
      if (i > 0) {
        b = new_body(b, i + 1 == js.size() ? name : "");
        if (b < 0) return false;
      }
      d->jnt_type[b] = js[i].type;
      for (int t = 0; t < 3; ++t) {
        d->axis[b][t] = js[i].axis[t];
        d->jnt_pos[b][t] = js[i].pos[t];
      }
      d->armature[b] = js[i].armature;
    }
    bool inertial = false;
    MassProps from_geoms;
    int ngeom = 0;
    for (const auto& kp : n.kids) {
      const XNode& k = *kp;
      if (k.tag == "inertial") {
        inertial = true;
        double m = 0;
        if (!nums(k.get("mass"), &m, 1)) return fail("inertial without mass");
        d->mass[b] = m;
        if (k.get("pos") && !nums(k.get("pos"), d->ipos[b], 3)) return fail("bad inertial pos");
        Quat iq;
        if (!orientation(k, nullptr, &iq)) return false;
        if (const std::string* fi = k.get("fullinertia")) {
          double v[6];
          if (!nums(fi, v, 6)) return fail("bad fullinertia");
          const double A[9] = {v[0], v[3], v[4], v[3], v[1], v[5], v[4], v[5], v[2]};
          double lam[3], V[9];
          eig3(A, lam, V);
          // right-handed principal frame
          const double det = V[0] * (V[4] * V[8] - V[5] * V[7]) - V[1] * (V[3] * V[8] - V[5] * V[6]) +
                             V[2] * (V[3] * V[7] - V[4] * V[6]);
          if (det < 0)
            for (int i = 0; i < 3; ++i) V[3 * i + 2] = -V[3 * i + 2];
          const Quat pq = mat2quat(V);
          iq = qnorm(qmul(iq, pq));
          for (int i = 0; i < 3; ++i) d->inertia[b][i] = lam[i];
        } else if (!nums(k.get("diaginertia"), d->inertia[b], 3)) {
          return fail("inertial needs diaginertia or fullinertia");
        }
        d->iquat[b][0] = iq.w; d->iquat[b][1] = iq.x; d->iquat[b][2] = iq.y; d->iquat[b][3] = iq.z;
      } else if (k.tag == "site") {
        if (!site(k, b, active)) return false;
      } else if (k.tag == "geom") {
        // mass properties are needed only under inertiafromgeom true, or auto without <inertial>
        // (decided below); an unsupported geom is an error only if it would be used
        if (comp.inertiafromgeom == 0) continue;
        MassProps g;
        bool used = false;
        if (!geom_mass(k, active, &g, &used)) {
          if (comp.inertiafromgeom == 1 || !has_inertial(n)) return false;
          err.clear();
          continue;
        }
        if (used) {
          mass_add(&from_geoms, g);
          ++ngeom;
        }
      } else if (k.tag == "frame" || k.tag == "include" || k.tag == "replicate" ||
                 k.tag == "composite" || k.tag == "flexcomp") {
        return fail("unsupported <" + k.tag + "> in body " + name);
      }
    }
    if (ngeom > 0 && (comp.inertiafromgeom == 1 || (comp.inertiafromgeom == 2 && !inertial)))
      set_inertia(b, from_geoms);
    for (const auto& kp : n.kids)
      if (kp->tag == "body" && !body(*kp, b, active)) return false;
    return true;
  }

  static bool has_inertial(const XNode& n) {
    for (const auto& kp : n.kids)
      if (kp->tag == "inertial") return true;
    return false;
  }

  bool site(const XNode& k, int b, const DefaultClass* active) {
    const DefaultClass* c = cls_of(k, active);
    if (!err.empty()) return false;
    Site s;
    const std::string* nm = k.get("name");
    s.name = nm ? *nm : "";
    s.body = b;
    s.pos[0] = s.pos[1] = s.pos[2] = 0.0;
    if (const std::string* ft = attr(k, c, "fromto")) {   // capsule-style site: its midpoint
      double v[6];
      if (!nums(ft, v, 6)) return fail("bad site fromto");
      for (int i = 0; i < 3; ++i) s.pos[i] = 0.5 * (v[i] + v[3 + i]);
    } else if (const std::string* p = attr(k, c, "pos")) {
      if (!nums(p, s.pos, 3)) return fail("bad site pos");
    }
    sites.push_back(s);
    return true;
  }

  bool model(const XNode& root) {
    const XNode* mj = nullptr;
    for (const auto& k : root.kids)
      if (k->tag == "mujoco") mj = k.get();
    if (!mj) return fail("no <mujoco> element");
    // compiler, option and defaults first (MuJoCo applies them regardless of their position)
    for (const auto& kp : mj->kids) {
      const XNode& k = *kp;
      if (k.tag == "compiler") {
        if (const std::string* a = k.get("angle")) {
          if (*a == "radian") comp.degree = false;
          else if (*a == "degree") comp.degree = true;
          else return fail("bad compiler angle");
        }
        if (const std::string* e = k.get("eulerseq")) comp.eulerseq = *e;
        if (const std::string* ig = k.get("inertiafromgeom")) {
          if (*ig == "false") comp.inertiafromgeom = 0;
          else if (*ig == "true") comp.inertiafromgeom = 1;
          else if (*ig == "auto") comp.inertiafromgeom = 2;
          else return fail("bad compiler inertiafromgeom");
        }
        if (const std::string* gr = k.get("inertiagrouprange")) {
          double v[2];
          if (!nums(gr, v, 2)) return fail("bad compiler inertiagrouprange");
          comp.group_lo = static_cast<int>(v[0]);
          comp.group_hi = static_cast<int>(v[1]);
        }
        // options that rescale or clamp masses are not modelled: refused rather than ignored
        for (const char* a : {"settotalmass", "boundmass", "boundinertia"})
          if (const std::string* v = k.get(a)) {
            double x = 0.0;
            if (!nums(v, &x, 1) || (std::strcmp(a, "settotalmass") == 0 ? x > 0.0 : x != 0.0))
              return fail(std::string("compiler ") + a + " unsupported");
          }
      } else if (k.tag == "option") {
        if (k.get("gravity") && !nums(k.get("gravity"), d->gravity, 3)) return fail("bad gravity");
      } else if (k.tag == "default") {
        if (!read_defaults(k, nullptr)) return false;
      }
    }
    if (!classes.count("main")) classes["main"] = std::make_unique<DefaultClass>();
    const DefaultClass* main_cls = classes["main"].get();
    int nworld = 0;
    for (const auto& kp : mj->kids) {
      if (kp->tag != "worldbody") continue;
      ++nworld;
      for (const auto& bp : kp->kids) {
        if (bp->tag == "body") {
          if (!body(*bp, -1, main_cls)) return false;
        } else if (bp->tag == "site") {
          if (!site(*bp, -1, main_cls)) return false;
        } else if (bp->tag == "frame" || bp->tag == "replicate") {
          return fail("unsupported <" + bp->tag + "> in worldbody");
        }
      }
    }
    if (nworld == 0) return fail("no <worldbody>");
    if (d->nbody == 0) return fail("no bodies");
    // MuJoCo numbers sites in body order (world first, then bodies depth-first); a stable sort
    // by body keeps document order within a body
    std::vector<Site> ordered;
    for (int b = -1; b < d->nbody; ++b)
      for (const Site& s : sites)
        if (s.body == b) ordered.push_back(s);
    sites.swap(ordered);
    return true;
  }

  // Welded (joint-less) non-root bodies are fused into their parents, as MuJoCo's
  // <compiler fusestatic="true"> does: their children and sites move into the parent's frame and
  // their mass and inertia are added to the parent's about the combined COM (re-diagonalised).
  // mj_fullM, qfrc_bias and every site Jacobian are unchanged mathematically; names of fused
  // bodies resolve to the body they were fused into (mj_jac of a welded body = its parent's).
  bool fuse_and_emit(osc_kin_desc* out) {
    const int nb = d->nbody;
    std::vector<int> alias(nb), keep(nb, 1);
    for (int b = 0; b < nb; ++b) alias[b] = b;
    for (int b = nb - 1; b >= 0; --b) {
      const int p = d->parent[b];
      if (d->jnt_type[b] != OSC_KIN_JOINT_NONE || p < 0) continue;
      double R[9];
      quat2mat(d->quat[b], R);
      auto to_parent = [&](const double* v, double* o) {
        for (int i = 0; i < 3; ++i)
          o[i] = d->pos[b][i] + R[3 * i] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
      };
      const Quat qb{d->quat[b][0], d->quat[b][1], d->quat[b][2], d->quat[b][3]};
      for (int c = b + 1; c < nb; ++c) {
        if (!keep[c] || d->parent[c] != b) continue;
        double np[3];
        to_parent(d->pos[c], np);
        for (int i = 0; i < 3; ++i) d->pos[c][i] = np[i];
        const Quat qc = qnorm(qmul(qb, {d->quat[c][0], d->quat[c][1], d->quat[c][2], d->quat[c][3]}));
        d->quat[c][0] = qc.w; d->quat[c][1] = qc.x; d->quat[c][2] = qc.y; d->quat[c][3] = qc.z;
        d->parent[c] = p;
      }
      for (Site& st : sites) {
        if (st.body != b) continue;
        double np[3];
        to_parent(st.pos, np);
        for (int i = 0; i < 3; ++i) st.pos[i] = np[i];
        st.body = p;
      }
      if (d->mass[b] > 0.0) {   // composite inertia about the combined COM, parent frame
        const double m1 = d->mass[p], m2 = d->mass[b], m = m1 + m2;
        double c2[3], Rib[9], Rw[9], Ri1[9], I[9] = {0};
        to_parent(d->ipos[b], c2);
        quat2mat(d->iquat[b], Rib);
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) {
            double t = 0.0;
            for (int k = 0; k < 3; ++k) t += R[3 * i + k] * Rib[3 * k + j];
            Rw[3 * i + j] = t;
          }
        quat2mat(d->iquat[p], Ri1);
        double c[3];
        for (int i = 0; i < 3; ++i) c[i] = (m1 * d->ipos[p][i] + m2 * c2[i]) / m;
        auto add = [&](const double* Rr, const double* diag, double mass, const double* com) {
          double dv[3] = {com[0] - c[0], com[1] - c[1], com[2] - c[2]};
          const double dd = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
          for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
              double t = 0.0;
              for (int k = 0; k < 3; ++k) t += Rr[3 * i + k] * diag[k] * Rr[3 * j + k];
              I[3 * i + j] += t + mass * ((i == j ? dd : 0.0) - dv[i] * dv[j]);
            }
        };
        add(Ri1, d->inertia[p], m1, d->ipos[p]);
        add(Rw, d->inertia[b], m2, c2);
        double lam[3], V[9];
        eig3(I, lam, V);
        const double det = V[0] * (V[4] * V[8] - V[5] * V[7]) - V[1] * (V[3] * V[8] - V[5] * V[6]) +
                           V[2] * (V[3] * V[7] - V[4] * V[6]);
        if (det < 0)
          for (int i = 0; i < 3; ++i) V[3 * i + 2] = -V[3 * i + 2];
        const Quat iq = mat2quat(V);
        d->mass[p] = m;
        for (int i = 0; i < 3; ++i) {
          d->ipos[p][i] = c[i];
          d->inertia[p][i] = lam[i] < 0.0 ? 0.0 : lam[i];
        }
        d->iquat[p][0] = iq.w; d->iquat[p][1] = iq.x; d->iquat[p][2] = iq.y; d->iquat[p][3] = iq.z;
      }
      keep[b] = 0;
      alias[b] = p;
    }
    std::vector<int> newid(nb, -1);
    int n = 0;
    for (int b = 0; b < nb; ++b)
      if (keep[b]) newid[b] = n++;
    if (n > OSC_KIN_MAX_BODIES) return fail("too many bodies after fusing welded bodies");
    final_id.assign(nb, -1);
    for (int b = 0; b < nb; ++b) {
      int a = b;
      while (!keep[a]) a = alias[a];
      final_id[b] = newid[a];
    }
    std::memset(out, 0, sizeof(*out));
    out->nbody = n;
    for (int i = 0; i < 3; ++i) out->gravity[i] = d->gravity[i];
    for (int b = 0; b < nb; ++b) {
      if (!keep[b]) continue;
      const int o = newid[b];
      out->parent[o] = d->parent[b] < 0 ? -1 : final_id[d->parent[b]];
      out->jnt_type[o] = d->jnt_type[b];
      std::memcpy(out->pos[o], d->pos[b], sizeof(out->pos[o]));
      std::memcpy(out->quat[o], d->quat[b], sizeof(out->quat[o]));
      std::memcpy(out->axis[o], d->axis[b], sizeof(out->axis[o]));
      std::memcpy(out->jnt_pos[o], d->jnt_pos[b], sizeof(out->jnt_pos[o]));
      out->armature[o] = d->armature[b];
      out->mass[o] = d->mass[b];
      std::memcpy(out->ipos[o], d->ipos[b], sizeof(out->ipos[o]));
      std::memcpy(out->iquat[o], d->iquat[b], sizeof(out->iquat[o]));
      std::memcpy(out->inertia[o], d->inertia[b], sizeof(out->inertia[o]));
    }
    for (Site& st : sites)
      if (st.body >= 0) st.body = final_id[st.body];
    return true;
  }
  std::vector<int> final_id;   // raw body -> emitted body
};

}  // namespace

extern "C" int osc_kin_desc_from_mjcf(const char* xml_path, const char* const* body_names,
                                      const char* const* site_names, int32_t nsite,
                                      int32_t site_order, osc_kin_desc* desc) {
  if (!xml_path || !desc || nsite < 1 || nsite > OSC_KIN_MAX_SITES || !body_names ||
      (site_order == OSC_MJCF_SITES_BY_NAME && !site_names) ||
      (site_order != OSC_MJCF_SITES_BY_NAME && site_order != OSC_MJCF_SITES_MODEL_ORDER))
    return OSC_ERR_INVALID_ARGUMENT;
  std::string text;
  if (!read_text(xml_path, &text)) {
    std::fprintf(stderr, "osc_kin_desc_from_mjcf: cannot open %s\n", xml_path);
    return OSC_ERR_IO;
  }
  std::string err;
  XmlParser parser(text);
  std::unique_ptr<XNode> root = parser.parse(&err);
  if (root) {
    const std::string xp(xml_path);
    const size_t slash = xp.rfind('/');
    if (!expand_includes(root.get(), slash == std::string::npos ? "." : xp.substr(0, slash), 0, &err))
      root.reset();
  }
  Loader L;
  auto raw = std::make_unique<RawDesc>();
  L.d = raw.get();
  if (!root || !L.model(*root) || !L.fuse_and_emit(desc)) {
    std::fprintf(stderr, "osc_kin_desc_from_mjcf: %s: %s\n", xml_path, (root ? L.err : err).c_str());
    std::memset(desc, 0, sizeof(*desc));
    return OSC_ERR_IO;
  }
  // task sites (operational_space_controller.h:125-152 name lookups; :373 / W :417 point rows)
  auto body_id = [&](const char* name) {
    for (int b = 0; b < static_cast<int>(L.body_name.size()); ++b)
      if (name && L.body_name[b] == name) return L.final_id[b];
    return -1;
  };
  desc->nsite = nsite;
  desc->has_jac_body = 1;
  for (int k = 0; k < nsite; ++k) {
    const int jb = body_id(body_names[k]);
    int si = -1;
    if (site_order == OSC_MJCF_SITES_MODEL_ORDER) {
      si = k < static_cast<int>(L.sites.size()) ? k : -1;
    } else {
      for (int i = 0; i < static_cast<int>(L.sites.size()); ++i)
        if (site_names[k] && L.sites[i].name == site_names[k]) si = i;
    }
    const bool world_site = si >= 0 && L.sites[si].body < 0;
    if (jb < 0 || si < 0 || world_site) {
      std::fprintf(stderr, "osc_kin_desc_from_mjcf: %s: task site %d: %s\n", xml_path, k,
                   jb < 0 ? "body not found" : world_site ? "world site unsupported" : "site not found");
      std::memset(desc, 0, sizeof(*desc));
      return OSC_ERR_IO;
    }
    desc->site_body[k] = L.sites[si].body;
    for (int i = 0; i < 3; ++i) desc->site_pos[k][i] = L.sites[si].pos[i];
    desc->site_jac_body[k] = jb;
  }
  return OSC_OK;
}

extern "C" int osc_kin_desc_from_mjcf_robot(const char* robot, const char* yaml_path,
                                            const char* xml_path, osc_kin_desc* desc) {
  if (!robot || !xml_path || !desc) return OSC_ERR_INVALID_ARGUMENT;
  std::vector<std::string> bodies, sites;
  const int rc = osc_config_lists(robot, yaml_path, &bodies, &sites);
  if (rc != OSC_OK) return rc;
  std::vector<const char*> bn, sn;
  for (const auto& s : bodies) bn.push_back(s.c_str());
  for (const auto& s : sites) sn.push_back(s.c_str());
  // the Go2 controller reads site_xpos rows in model order (G/osc.h:373); WaLTER's re-indexes
  // them by the configured site ids (W/osc.h:417)
  const int order = std::strcmp(robot, "unitree_go2") == 0 ? OSC_MJCF_SITES_MODEL_ORDER
                                                           : OSC_MJCF_SITES_BY_NAME;
  return osc_kin_desc_from_mjcf(xml_path, bn.data(), sn.data(), static_cast<int32_t>(sn.size()),
                                order, desc);
}
