// osc_model.cpp -- host side of the model descriptor: robot registry + run-time YAML loader.
//
// The reference bakes the YAML (weights, friction, site lists) into CasADi-generated C at
// build time (unitree_go2/autogen/autogen.py:19-56, :362-411) and hard-codes the bound
// vectors in each controller header (unitree_go2/operational_space_controller.h:276-309,
// walter_sr/operational_space_controller.h:309-353).  Here the same YAML schema is read at
// run time into an osc_model_desc, so the alternative WaLTER weight sets under
// config/walter_sr/*.yaml load without a rebuild.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include <dlfcn.h>

#include "osc_batch.h"

namespace {

struct RobotInfo {
  const char* name;
  int nv, nu, nc;
  std::vector<std::string> site_keys;   // weight-key prefix per site, in site order
  std::vector<double> u_lb, u_ub;
  const char* default_config;
};

// Site-key order = the order autogen.py splits the task rows into sites:
//   unitree_go2/autogen/autogen.py:160-219 ; walter_sr/autogen/autogen.py:163-330.
const std::vector<RobotInfo>& registry() {
  static const std::vector<RobotInfo> robots = [] {
    std::vector<RobotInfo> r;
    std::vector<double> go2_ub = {23.7, 23.7, 45.3, 23.7, 23.7, 45.3,
                                  23.7, 23.7, 45.3, 23.7, 23.7, 45.3};   // osc.h:291-296
    std::vector<double> go2_lb;
    for (double v : go2_ub) go2_lb.push_back(-v);                         // osc.h:285-290
    r.push_back({"unitree_go2", 18, 12, 4, {"base", "fr", "fl", "hr", "hl"}, go2_lb, go2_ub,
                 "unitree_go2_config.yaml"});
    std::vector<std::string> walter_keys = {"torso", "tls", "trs", "hls", "hrs", "tlh",
                                            "trh", "hlh", "hrh", "tlf", "tlr", "trf",
                                            "trr", "hlf", "hlr", "hrf", "hrr"};
    std::vector<double> w_lb(8, -1000.0), w_ub(8, 1000.0);               // walter osc.h:309-320
    r.push_back({"walter_sr", 14, 8, 8, walter_keys, w_lb, w_ub, "walter_sr_config.yaml"});
    r.push_back({"walter_sr_wheels", 14, 8, 8, walter_keys, w_lb, w_ub,
                 "walter_sr_wheels_config.yaml"});
    return r;
  }();
  return robots;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

std::string strip_comment(const std::string& s) {
  size_t p = s.find('#');
  return p == std::string::npos ? s : s.substr(0, p);
}

// Minimal YAML reader for the reference config schema: top-level keys holding a block list
// ("- item"), an inline list ("[a, b]"), a scalar, or a one-level mapping of scalars.
struct MiniYaml {
  std::map<std::string, std::vector<std::string>> lists;
  std::map<std::string, std::string> scalars;
  std::map<std::string, std::map<std::string, std::string>> maps;

  bool parse(std::istream& in, std::string* err) {
    std::string line, cur;
    bool cur_inline_open = false;
    std::string inline_buf;
    int lineno = 0;
    while (std::getline(in, line)) {
      ++lineno;
      std::string raw = strip_comment(line);
      if (trim(raw).empty()) continue;
      size_t indent = raw.find_first_not_of(" \t");
      std::string body = trim(raw);
      if (cur_inline_open) {                      // continuation of "[a, b,\n c]"
        inline_buf += " " + body;
        if (body.find(']') != std::string::npos) {
          cur_inline_open = false;
          split_inline(cur, inline_buf);
        }
        continue;
      }
      if (indent == 0) {
        size_t colon = body.find(':');
        if (colon == std::string::npos) {
          *err = "line " + std::to_string(lineno) + ": expected 'key:'";
          return false;
        }
        cur = trim(body.substr(0, colon));
        std::string rest = trim(body.substr(colon + 1));
        if (rest.empty()) continue;               // block list or mapping follows
        if (rest[0] == '[') {
          inline_buf = rest;
          if (rest.find(']') == std::string::npos) {
            cur_inline_open = true;
          } else {
            split_inline(cur, inline_buf);
          }
        } else {
          scalars[cur] = rest;
        }
        continue;
      }
      if (cur.empty()) {
        *err = "line " + std::to_string(lineno) + ": indented entry without a key";
        return false;
      }
      if (body[0] == '-') {
        lists[cur].push_back(trim(body.substr(1)));
      } else {
        size_t colon = body.find(':');
        if (colon == std::string::npos) {
          *err = "line " + std::to_string(lineno) + ": expected 'name: value'";
          return false;
        }
        maps[cur][trim(body.substr(0, colon))] = trim(body.substr(colon + 1));
      }
    }
    return true;
  }

  void split_inline(const std::string& key, const std::string& buf) {
    size_t a = buf.find('['), b = buf.rfind(']');
    std::string inner = buf.substr(a + 1, b - a - 1);
    std::stringstream ss(inner);
    std::string item;
    auto& v = lists[key];
    while (std::getline(ss, item, ',')) {
      item = trim(item);
      if (!item.empty()) v.push_back(item);
    }
  }
};

bool to_double(const std::string& s, double* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  double v = std::strtod(s.c_str(), &end);
  if (end == s.c_str() || trim(std::string(end)).size() != 0) return false;
  *out = v;
  return true;
}

std::string library_dir() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&osc_desc_from_yaml), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s);
  }
  return ".";
}

}  // namespace

extern "C" int osc_desc_from_yaml(const char* robot, const char* yaml_path, osc_model_desc* desc) {
  if (!robot || !desc) return OSC_ERR_INVALID_ARGUMENT;
  const RobotInfo* info = nullptr;
  for (const auto& r : registry())
    if (std::strcmp(r.name, robot) == 0) info = &r;
  if (!info) return OSC_ERR_INVALID_ARGUMENT;

  std::string path = yaml_path ? std::string(yaml_path)
                               : library_dir() + "/../config/" + info->default_config;
  std::ifstream in(path);
  if (!in) return OSC_ERR_IO;
  MiniYaml y;
  std::string err;
  if (!y.parse(in, &err)) {
    std::fprintf(stderr, "osc_desc_from_yaml: %s: %s\n", path.c_str(), err.c_str());
    return OSC_ERR_IO;
  }
  const auto& noncontact = y.lists["noncontact_site_list"];
  const auto& contact = y.lists["contact_site_list"];
  const auto& bodies = y.lists["body_list"];
  int ns = static_cast<int>(noncontact.size() + contact.size());
  // autogen.py:42 -- one body per site; sizes must match the robot's generated layout.
  if (ns != static_cast<int>(bodies.size()) || ns != static_cast<int>(info->site_keys.size()) ||
      static_cast<int>(contact.size()) != info->nc) {
    std::fprintf(stderr, "osc_desc_from_yaml: %s: site/body lists do not match robot %s\n",
                 path.c_str(), robot);
    return OSC_ERR_IO;
  }
  std::memset(desc, 0, sizeof(*desc));
  desc->nv = info->nv;
  desc->nu = info->nu;
  desc->nc = info->nc;
  desc->ns = ns;
  if (!to_double(y.scalars["friction_coefficient"], &desc->mu)) return OSC_ERR_IO;
  auto& w = y.maps["weights_config"];
  for (int i = 0; i < ns; ++i) {
    const std::string& k = info->site_keys[i];
    if (!to_double(w[k + "_translational_tracking"], &desc->w_pos[i])) return OSC_ERR_IO;
    if (!to_double(w[k + "_rotational_tracking"], &desc->w_rot[i])) return OSC_ERR_IO;
  }
  if (!to_double(w["torque"], &desc->w_torque)) return OSC_ERR_IO;
  if (!to_double(w["regularization"], &desc->w_reg)) return OSC_ERR_IO;
  for (int i = 0; i < info->nu; ++i) {
    desc->u_lb[i] = info->u_lb[i];
    desc->u_ub[i] = info->u_ub[i];
  }
  const double inf = 1e30;                    // OSQP_INFTY (osqp 0.6.3 constants.h)
  const double big_number = 1e4;              // `const float big_number = 1e4;` osc.h:279
  desc->z_lb[0] = -inf; desc->z_lb[1] = -inf; desc->z_lb[2] = 0.0;
  desc->z_ub[0] = inf;  desc->z_ub[1] = inf;  desc->z_ub[2] = big_number;
  desc->infinity = inf;
  // interior-point stop.  The full-space refinement that follows (osc_ipm.hpp) needs only an
  // approximate active set: its rounds add the rows its point violates and drop the rows whose
  // multiplier comes out negative, and it is kept only at a KKT point.  So the
  // interior point stops early -- Go2 at 1e-6, WaLTER at 1e-8 (numpy model of the kernel,
  // tools/kkt_study.py, 1,024-env synthetic and joint-state batches: no rejection, worst error
  // vs the exact optimum 1e-11; slowest wave of four envs -1.5 (Go2) / -2.0 (WaLTER) iterations
  // for +0.0-0.7 (Go2) / +0.5-1.4 (WaLTER) refinement steps against 1e-9 / 1e-12).  The opt-in
  // wheel rows keep 1e-12: their rotated Newton systems stop on their own stall test
  // (DESIGN.md §3.1), and their refinement's acceptance bounds were set around that stop.
  desc->eps_mu = std::strcmp(robot, "unitree_go2") == 0 ? 1e-6 : 1e-8;   // (wheel rows: below)
  desc->max_iter = 50;   // normal solves take <= 24; the margin covers a re-centred stall
  // optional wheel no-slip rows (walter_sr_wheels/autogen/autogen.py:128-240, commented out
  // upstream): `wheel_no_slip: true`, `wheel_radius: r` (or one per wheel, the design's 0.065 at
  // :64), `wheel_dofs: [k_0, ...]` (the dof of each wheel's joint, the design's jnt_dofadr lookup
  // at :64-94; -1 = none).  Absent keys: off, the reference's QP.
  const std::string& ns_flag = y.scalars["wheel_no_slip"];
  if (ns_flag == "true" || ns_flag == "True" || ns_flag == "1") {
    desc->wheel_rows = 1;
    desc->eps_mu = 1e-12;   // the wheel rows' interior point keeps the late stop (above)
    // the active-set fallback (osc_gi_kernel) takes every env the interior point leaves at
    // max_iter, so the cap can sit just above the converging envs' 21 iterations: 2,048 tumbling
    // envs 5.34 -> 4.53 ms per solve, all OK and certified either way (profiles/r04w/)
    desc->max_iter = 25;
    const auto& rl = y.lists["wheel_radius"];
    double r = 0.0;
    const bool scalar_r = rl.empty() && to_double(y.scalars["wheel_radius"], &r);
    const auto& dl = y.lists["wheel_dofs"];
    if ((!scalar_r && static_cast<int>(rl.size()) != info->nc) ||
        static_cast<int>(dl.size()) != info->nc) {
      std::fprintf(stderr, "osc_desc_from_yaml: %s: wheel_radius / wheel_dofs need %d entries\n",
                   path.c_str(), info->nc);
      return OSC_ERR_IO;
    }
    for (int i = 0; i < info->nc; ++i) {
      double k = 0.0;
      if (!scalar_r && !to_double(rl[i], &r)) return OSC_ERR_IO;
      if (!to_double(dl[i], &k) || k != static_cast<int>(k) || k < -1 || k >= info->nv)
        return OSC_ERR_IO;
      desc->wheel_radius[i] = r;
      desc->wheel_dof[i] = static_cast<int32_t>(k);
    }
  } else if (!ns_flag.empty() && ns_flag != "false" && ns_flag != "False" && ns_flag != "0") {
    return OSC_ERR_IO;
  }
  return OSC_OK;
}

// The config's body_list and noncontact_site_list + contact_site_list (autogen.py:32-35), for the
// MJCF reader (osc_mjcf.cpp: osc_kin_desc_from_mjcf_robot).  Same file and checks as above.
int osc_config_lists(const char* robot, const char* yaml_path, std::vector<std::string>* bodies,
                     std::vector<std::string>* sites) {
  osc_model_desc d;
  int rc = osc_desc_from_yaml(robot, yaml_path, &d);   // validates the lists against the robot
  if (rc != OSC_OK) return rc;
  const RobotInfo* info = nullptr;
  for (const auto& r : registry())
    if (std::strcmp(r.name, robot) == 0) info = &r;
  std::string path = yaml_path ? std::string(yaml_path)
                               : library_dir() + "/../config/" + info->default_config;
  std::ifstream in(path);
  MiniYaml y;
  std::string err;
  if (!in || !y.parse(in, &err)) return OSC_ERR_IO;
  *bodies = y.lists["body_list"];
  *sites = y.lists["noncontact_site_list"];
  for (const auto& c : y.lists["contact_site_list"]) sites->push_back(c);
  return OSC_OK;
}

extern "C" const char* osc_status_string(int status) {
  switch (status) {
    case OSC_OK: return "OSC_OK";
    case OSC_ERR_INVALID_ARGUMENT: return "OSC_ERR_INVALID_ARGUMENT";
    case OSC_ERR_UNSUPPORTED_DIMS: return "OSC_ERR_UNSUPPORTED_DIMS";
    case OSC_ERR_IO: return "OSC_ERR_IO";
    case OSC_ERR_DEVICE: return "OSC_ERR_DEVICE";
    case OSC_ERR_NO_DEVICE: return "OSC_ERR_NO_DEVICE";
    default: return "OSC_ERR_UNKNOWN";
  }
}

extern "C" int osc_abi_version(void) { return OSC_ABI_VERSION; }
