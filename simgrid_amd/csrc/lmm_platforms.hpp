// lmm_platforms.hpp — fat-tree and dragonfly cluster platforms and the LMM systems their flows build
// (input generation only: no solver arithmetic here).  SURVEY.md §8 row f3.
//
// A platform is the set of links one <cluster topology="FAT_TREE"|"DRAGONFLY"> creates and the route
// between two of its hosts; a flow is one communication between two random hosts, turned into one
// LMM variable the way the network / ptask models do it:
//   * routing restates FatTreeZone.cpp:62-129 (d-mod-k up, label-matching down, including the way the
//     down loop keeps scanning the ports of the switch it just reached) and DragonflyZone.cpp:238-336
//     (minimal routing, including its flat router re-indexing);
//   * link creation follows sg_platf.cpp:130-139 (SPLITDUPLEX -> an _UP and a _DOWN link),
//     FatTreeZone.cpp:443-485, DragonflyZone.cpp:135-236 and the cluster's private loopback /
//     limiter links, sg_platf.cpp:214-251;
//   * flows restate network_cm02.cpp:165-279 (CM02 and LV08; LV08 = bandwidth factor 0.97 and
//     weight_S 20537, network_cm02.cpp:36-64; with crosstraffic the back route at weight 0.05) and
//     ptask_L07.cpp:143-208, 389-417 (L07: both CPUs at weight 0, the route's links at the flow size).
// Each flow is built in the state it has once its latency is paid (update_actions_state restores the
// penalty and sets the TCP-gamma bound, network_cm02.cpp:105-146, ptask_L07.cpp:89-98), so the
// generated system is a solve-ready snapshot of a running simulation.
//
// Only links a route can use get a constraint.  The reference also creates links no route of these
// zones reads (the cluster's per-host "_link_" and, for fat trees, the cluster-level loopbacks and the
// switches' loopbacks, ClusterZone.cpp:126-147, FatTreeZone.cpp:455-462): they would carry no element
// and change no value.
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "lmm_generators.hpp"

namespace lmm_plat {

enum Topology { FAT_TREE = 0, DRAGONFLY = 1 };
enum LinkPolicy { SHARED = 0, SPLITDUPLEX = 1, FATPIPE = 2 };
enum FlowModel { CM02 = 0, LV08 = 1, L07 = 2 };

struct Params {
  int topology = FAT_TREE;
  std::string topo;                   // topo_parameters
  double bw = 1.25e8, lat = 5e-5;     // examples/platforms/cluster_*.xml: bw="125MBps" lat="50us"
  int policy = SPLITDUPLEX;           // the cluster's default sharing policy
  double loopback_bw = 0.0, loopback_lat = 0.0, limiter_bw = 0.0;
  double speed = 1e9;                 // host speed, "1Gf" (L07 CPU constraints)
  int model = LV08;
  int64_t n_flows = 1000;
  uint64_t seed = 1;
  double size_min = 1e6, size_max = 1e9;  // L07 flow sizes (bytes), uniform
  double tcp_gamma = 4194304.0;       // network/TCP-gamma default
  bool crosstraffic = true;           // network/crosstraffic default
};

// From any struct with the fields of lmm_platform_params (include/lmm/lmm_system.h).
template <class C>
Params params_from(const C& c) {
  Params p;
  p.topology = c.topology;
  p.topo = c.topo_parameters ? c.topo_parameters : "";
  p.bw = c.bw;
  p.lat = c.lat;
  p.policy = c.policy;
  p.loopback_bw = c.loopback_bw;
  p.loopback_lat = c.loopback_lat;
  p.limiter_bw = c.limiter_bw;
  p.speed = c.speed;
  p.model = c.model;
  p.crosstraffic = c.crosstraffic != 0;
  p.n_flows = c.n_flows;
  p.seed = c.seed;
  p.size_min = c.size_min;
  p.size_max = c.size_max;
  p.tcp_gamma = c.tcp_gamma;
  if (p.policy < SHARED || p.policy > FATPIPE)
    throw std::invalid_argument("unknown sharing policy " + std::to_string(p.policy));
  if (p.n_flows < 0)
    throw std::invalid_argument("negative flow count");
  return p;
}

struct Link {
  double bw, lat;
  bool fatpipe;
  // WIFI access point (NetworkWifiLink, network_cm02.cpp:383-420): the rates of the flow's source and destination
  // stations on it (get_host_rate: -1 = not associated); bw / lat are then the link's own (1 / bandwidth factor, 0)
  bool wifi = false;
  double src_rate = -1.0, dst_rate = -1.0;
};

inline std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out(1);
  for (char ch : s) {
    if (ch == sep)
      out.emplace_back();
    else
      out.back() += ch;
  }
  return out;
}

inline int to_int(const std::string& s, const std::string& what) {
  int v = 0;
  try {
    v = std::stoi(s);
  } catch (const std::exception&) {
    throw std::invalid_argument(what + s);
  }
  if (v <= 0)
    throw std::invalid_argument(what + s);
  return v;
}

class Platform {
 public:
  std::vector<Link> links;
  int n_hosts = 0;
  virtual ~Platform() = default;
  // links of the route src -> dst in route order; adds their latency to *lat when lat is given
  virtual void route(int src, int dst, std::vector<int>& out, double* lat) const = 0;

 protected:
  // sg_platf.cpp:130-139: a SPLITDUPLEX link is an _UP and a _DOWN link; returns (up, down)
  std::pair<int, int> new_link(double bw, double lat, int policy) {
    const int up = int(links.size());
    links.push_back({bw, lat, policy == FATPIPE});
    if (policy != SPLITDUPLEX)
      return {up, up};
    links.push_back({bw, lat, false});
    return {up, up + 1};
  }
  void add_lat(int l, double* lat) const {
    if (lat)
      *lat += links[size_t(l)].lat;
  }
};

// ---- FatTreeZone.cpp ----
class FatTree : public Platform {
  struct Node {
    int level = 0, position = 0;
    std::vector<int> label, parents, children;  // parents / children: cable id per port, -1 = none
    int loopback = -1, limiter = -1;
  };
  struct Cable {
    int up_node, down_node, up_link, down_link;
  };
  int levels_ = 0;
  std::vector<int> down_, up_, ports_, by_level_;
  std::vector<Node> nodes_;  // hosts (level 0, by position), then switches level by level
  std::vector<Cable> cables_;
  bool has_loopback_ = false, has_limiter_ = false;

  int level_start(int level) const {
    int k = 0;
    for (int i = 0; i < level; i++)
      k += by_level_[size_t(i)];
    return k;
  }
  // FatTreeZone.cpp:204-234
  bool related(const Node& parent, const Node& child) const {
    if (parent.level != child.level + 1)
      return false;
    for (int i = 0; i < levels_; i++)
      if (parent.label[size_t(i)] != child.label[size_t(i)] && i + 1 != parent.level)
        return false;
    return true;
  }
  // FatTreeZone.cpp:41-60
  bool in_sub_tree(const Node& root, const Node& node) const {
    if (root.level <= node.level)
      return false;
    for (int i = 0; i < node.level; i++)
      if (root.label[size_t(i)] != node.label[size_t(i)])
        return false;
    for (int i = root.level; i < levels_; i++)
      if (root.label[size_t(i)] != node.label[size_t(i)])
        return false;
    return true;
  }

 public:
  explicit FatTree(const Params& p) {
    const std::string msg =
        "Fat trees are defined by the levels number and 3 vectors, see the documentation for more information";
    const auto parts = split(p.topo, ';');
    if (parts.size() != 4)
      throw std::invalid_argument(msg);
    levels_ = to_int(parts[0], "First parameter is not the amount of levels:");
    const char* what[3] = {"Invalid lower level node number:", "Invalid upper level node number:",
                           "Invalid lower level port number:"};
    std::vector<int>* vecs[3] = {&down_, &up_, &ports_};
    for (int k = 0; k < 3; k++) {
      const auto t = split(parts[size_t(k) + 1], ',');
      if (int(t.size()) != levels_)
        throw std::invalid_argument(msg);
      for (const auto& x : t)
        vecs[k]->push_back(to_int(x, what[k]));
    }
    has_loopback_ = p.loopback_bw > 0 || p.loopback_lat > 0;
    has_limiter_ = p.limiter_bw > 0;
    // FatTreeNode's constructor pushes both bandwidths into one link template (FatTreeZone.cpp:446-462)
    // and the network model refuses a non-wifi link with two bandwidths (network_cm02.cpp:99)
    if (has_loopback_ && has_limiter_)
      throw std::invalid_argument("Non WIFI links must use only 1 bandwidth.");

    // FatTreeZone.cpp:236-262
    by_level_.assign(size_t(levels_) + 1, 1);
    for (int i = 0; i < levels_; i++)
      by_level_[0] *= down_[size_t(i)];
    for (int i = 0; i < levels_; i++) {
      int n = 1;
      for (int j = 0; j <= i; j++)
        n *= up_[size_t(j)];
      for (int j = i + 1; j < levels_; j++)
        n *= down_[size_t(j)];
      by_level_[size_t(i) + 1] = n;
    }
    n_hosts = by_level_[0];
    // hosts with their private links (add_processing_node, FatTreeZone.cpp:337-347, 443-463)
    for (int h = 0; h < n_hosts; h++) {
      Node n;
      n.position = h;
      n.label.assign(size_t(levels_), 0);
      n.parents.assign(size_t(up_[0] * ports_[0]), -1);
      if (has_limiter_)
        n.limiter = new_link(p.limiter_bw, 0.0, SHARED).first;
      if (has_loopback_)
        n.loopback = new_link(p.loopback_bw, p.loopback_lat, FATPIPE).first;
      nodes_.push_back(std::move(n));
    }
    // switches (FatTreeZone.cpp:264-277); their limiters are on the routes, their loopbacks are not
    for (int i = 0; i < levels_; i++)
      for (int j = 0; j < by_level_[size_t(i) + 1]; j++) {
        Node n;
        n.level = i + 1;
        n.position = j;
        n.label.assign(size_t(levels_), 0);
        n.children.assign(size_t(down_[size_t(i)] * ports_[size_t(i)]), -1);
        if (i != levels_ - 1)
          n.parents.assign(size_t(up_[size_t(i) + 1] * ports_[size_t(i) + 1]), -1);
        if (has_limiter_)
          n.limiter = new_link(p.limiter_bw, 0.0, SHARED).first;
        nodes_.push_back(std::move(n));
      }
    // labels: mixed-radix counters per level (FatTreeZone.cpp:280-324)
    std::vector<int> maxl(static_cast<size_t>(levels_)), cur(static_cast<size_t>(levels_));
    size_t k = 0;
    for (int i = 0; i <= levels_; i++) {
      std::fill(cur.begin(), cur.end(), 0);
      for (int j = 0; j < levels_; j++)
        maxl[size_t(j)] = j + 1 > i ? down_[size_t(j)] : up_[size_t(j)];
      for (int j = 0; j < by_level_[size_t(i)]; j++, k++) {
        nodes_[k].label = cur;
        for (int pos = 0; pos < levels_; pos++) {
          if (++cur[size_t(pos)] < maxl[size_t(pos)])
            break;
          cur[size_t(pos)] = 0;
        }
      }
    }
    // cables, node by node in (level, position) order (FatTreeZone.cpp:161-202, 349-359, 465-485)
    k = 0;
    for (int i = 0; i < levels_; i++)
      for (int j = 0; j < by_level_[size_t(i)]; j++, k++) {
        const int level = nodes_[k].level;
        const int first = level_start(level + 1);
        for (int q = 0; q < by_level_[size_t(level) + 1]; q++) {
          const size_t pa = size_t(first + q);
          if (!related(nodes_[pa], nodes_[k]))
            continue;
          for (int port = 0; port < ports_[size_t(level)]; port++) {
            const int pport = nodes_[k].label[size_t(level)] + port * down_[size_t(level)];
            const int cport = nodes_[pa].label[size_t(level)] + port * up_[size_t(level)];
            const auto ud = new_link(p.bw, p.lat, p.policy);
            const int id = int(cables_.size());
            cables_.push_back({int(pa), int(k), ud.first, ud.second});
            nodes_[pa].children.at(size_t(pport)) = id;
            nodes_[k].parents.at(size_t(cport)) = id;
          }
        }
      }
  }

  void route(int src, int dst, std::vector<int>& out, double* lat) const override {
    const Node& d = nodes_[size_t(dst)];
    if (src == dst && has_loopback_) {
      out.push_back(nodes_[size_t(src)].loopback);
      add_lat(out.back(), lat);
      return;
    }
    size_t cur = size_t(src);
    while (!in_sub_tree(nodes_[cur], d)) {  // up: d-mod-k on the destination's position
      const Node& n = nodes_[cur];
      int x = d.position;
      for (int i = 0; i < n.level; i++)
        x /= up_[size_t(i)];
      x %= up_[size_t(n.level)];
      const int cb = n.parents.at(size_t(x));
      if (cb < 0)
        throw std::runtime_error("fat tree: missing up port");
      const Cable& c = cables_[size_t(cb)];
      out.push_back(c.up_link);
      add_lat(c.up_link, lat);
      if (has_limiter_)
        out.push_back(n.limiter);
      cur = size_t(c.up_node);
    }
    while (cur != size_t(dst)) {  // down: the port scan continues on the switch it just reached
      const size_t before = cur;
      for (size_t i = 0; i < nodes_[cur].children.size(); i++) {
        const Node& n = nodes_[cur];
        if (int(i) % down_[size_t(n.level) - 1] != d.label[size_t(n.level) - 1])
          continue;
        const int cb = n.children[i];
        if (cb < 0)
          throw std::runtime_error("fat tree: missing down port");
        const Cable& c = cables_[size_t(cb)];
        out.push_back(c.down_link);
        add_lat(c.down_link, lat);
        cur = size_t(c.down_node);
        if (has_limiter_)
          out.push_back(nodes_[cur].limiter);
      }
      if (cur == before)
        throw std::runtime_error("fat tree: no route down");
    }
  }
};

// ---- DragonflyZone.cpp ----
class Dragonfly : public Platform {
  struct Router {
    int group, chassis, blade;
    std::vector<int> my_nodes, green, black;
    int blue = -1;
  };
  int groups_ = 0, blue_ = 0, chassis_ = 0, black_ = 0, blades_ = 0, green_ = 0, nodes_ = 0, lpl_ = 1;
  bool has_loopback_ = false, has_limiter_ = false;
  std::vector<Router> routers_;
  std::vector<int> loopback_, limiter_;  // per host (the cluster's private links)

  const Router& router(size_t i) const {
    if (i >= routers_.size())
      throw std::out_of_range("dragonfly: router index out of range");
    return routers_[i];
  }
  static int link_at(const std::vector<int>& v, size_t i) {
    if (i >= v.size() || v[i] < 0)
      throw std::out_of_range("dragonfly: no such link");
    return v[i];
  }

 public:
  // rankId_to_coords (DragonflyZone.cpp:26-35): group, chassis, blade, node of host `rank`; pinned to the 120 lines
  // s4u-routing-get-clusters.tesh prints for cluster_dragonfly.xml (tests/test_platforms.py)
  void coords(int rank, int c[4]) const {
    const int per_group = chassis_ * blades_ * nodes_, per_chassis = blades_ * nodes_;
    c[0] = rank / per_group;
    rank %= per_group;
    c[1] = rank / per_chassis;
    rank %= per_chassis;
    c[2] = rank / nodes_;
    c[3] = rank % nodes_;
  }

  explicit Dragonfly(const Params& p) {
    const auto parts = split(p.topo, ';');
    if (parts.size() != 4)
      throw std::invalid_argument(
          "Dragonfly are defined by the number of groups, chassis per groups, blades per chassis, nodes per blade");
    const std::string lv =
        "Dragonfly topologies are defined by 3 levels with 2 elements each, and one with one element";
    int* dst[3][2] = {{&groups_, &blue_}, {&chassis_, &black_}, {&blades_, &green_}};
    const char* what[3][2] = {{"Invalid number of groups:", "Invalid number of links for the blue level:"},
                              {"Invalid number of groups:", "Invalid number of links for the black level:"},
                              {"Invalid number of groups:", "Invalid number of links for the green level:"}};
    for (int k = 0; k < 3; k++) {
      const auto t = split(parts[size_t(k)], ',');
      if (t.size() != 2)
        throw std::invalid_argument(lv);
      *dst[k][0] = to_int(t[0], what[k][0]);
      *dst[k][1] = to_int(t[1], what[k][1]);
    }
    nodes_ = to_int(parts[3], "Last parameter is not the amount of nodes per blade:");
    lpl_ = p.policy == SPLITDUPLEX ? 2 : 1;
    n_hosts = groups_ * chassis_ * blades_ * nodes_;
    has_loopback_ = p.loopback_bw > 0 || p.loopback_lat > 0;
    has_limiter_ = p.limiter_bw > 0;
    loopback_.assign(size_t(n_hosts), -1);
    limiter_.assign(size_t(n_hosts), -1);
    for (int h = 0; h < n_hosts; h++) {  // sg_platf.cpp:214-251
      if (has_loopback_)
        loopback_[size_t(h)] = new_link(p.loopback_bw, p.loopback_lat, FATPIPE).first;
      if (has_limiter_)
        limiter_[size_t(h)] = new_link(p.limiter_bw, 0.0, SHARED).first;
    }
    // DragonflyZone.cpp:126-133
    for (int i = 0; i < groups_; i++)
      for (int j = 0; j < chassis_; j++)
        for (int k = 0; k < blades_; k++)
          routers_.push_back(Router{i, j, k, std::vector<int>(size_t(lpl_ * nodes_), -1),
                                    std::vector<int>(size_t(blades_), -1), std::vector<int>(size_t(chassis_), -1)});
    const int n_routers = int(routers_.size());
    // DragonflyZone.cpp:158-236
    for (int i = 0; i < n_routers; i++)
      for (int j = 0; j < nodes_; j++) {
        const auto ud = new_link(p.bw, p.lat, p.policy);
        routers_[size_t(i)].my_nodes[size_t(j * lpl_)] = ud.first;
        if (lpl_ == 2)
          routers_[size_t(i)].my_nodes[size_t(j * lpl_ + 1)] = ud.second;
      }
    for (int i = 0; i < groups_ * chassis_; i++)
      for (int j = 0; j < blades_; j++)
        for (int k = j + 1; k < blades_; k++) {
          const auto ud = new_link(p.bw * green_, p.lat, p.policy);
          routers_[size_t(i * blades_ + j)].green[size_t(k)] = ud.first;
          routers_[size_t(i * blades_ + k)].green[size_t(j)] = ud.second;
        }
    for (int i = 0; i < groups_; i++)
      for (int j = 0; j < chassis_; j++)
        for (int k = j + 1; k < chassis_; k++)
          for (int l = 0; l < blades_; l++) {
            const auto ud = new_link(p.bw * black_, p.lat, p.policy);
            routers_[size_t(i * blades_ * chassis_ + j * blades_ + l)].black[size_t(k)] = ud.first;
            routers_[size_t(i * blades_ * chassis_ + k * blades_ + l)].black[size_t(j)] = ud.second;
          }
    for (int i = 0; i < groups_; i++)
      for (int j = i + 1; j < groups_; j++) {
        const size_t ri = size_t(i * blades_ * chassis_ + j), rj = size_t(j * blades_ * chassis_ + i);
        if (ri >= routers_.size() || rj >= routers_.size())
          throw std::invalid_argument("dragonfly: more groups than routers per group");
        const auto ud = new_link(p.bw * blue_, p.lat, p.policy);
        routers_[ri].blue = ud.first;
        routers_[rj].blue = ud.second;
      }
  }

  // DragonflyZone.cpp:238-336 (minimal routing; router indices computed as the reference does)
  void route(int src, int dst, std::vector<int>& out, double* lat) const override {
    if (src == dst && has_loopback_) {
      out.push_back(loopback_[size_t(src)]);
      add_lat(out.back(), lat);
      return;
    }
    int my[4], tg[4];
    coords(src, my);
    coords(dst, tg);
    const int cb = chassis_ * blades_;
    const size_t me = size_t(my[0] * cb + my[1] * blades_ + my[2]);
    const size_t target = size_t(tg[0] * cb + tg[1] * blades_ + tg[2]);
    size_t cur = me;
    auto hop = [&](int l) {
      out.push_back(l);
      add_lat(l, lat);
    };
    hop(link_at(router(me).my_nodes, size_t(my[3] * lpl_)));
    if (has_limiter_)
      out.push_back(limiter_[size_t(src)]);
    if (target != me) {
      if (router(target).group != router(cur).group) {
        if (router(cur).blade != tg[0]) {
          hop(link_at(router(cur).green, size_t(tg[0])));
          cur = size_t(my[0] * cb + my[1] * blades_ + tg[0]);
        }
        if (router(cur).chassis != 0) {
          hop(link_at(router(cur).black, 0));
          cur = size_t(my[0] * cb + tg[0]);
        }
        if (router(cur).blue < 0)
          throw std::out_of_range("dragonfly: no blue link");
        hop(router(cur).blue);
        cur = size_t(tg[0] * cb + my[0]);
      }
      if (router(target).blade != router(cur).blade) {
        hop(link_at(router(cur).green, size_t(tg[2])));
        cur = size_t(tg[0] * cb + tg[2]);
      }
      if (router(target).chassis != router(cur).chassis)
        hop(link_at(router(cur).black, size_t(tg[1])));
    }
    if (has_limiter_)
      out.push_back(limiter_[size_t(dst)]);
    hop(link_at(router(target).my_nodes, size_t(tg[3] * lpl_ + lpl_ - 1)));
  }
};

inline Platform* make_platform(const Params& p) {
  if (p.topology == FAT_TREE)
    return new FatTree(p);
  if (p.topology == DRAGONFLY)
    return new Dragonfly(p);
  throw std::invalid_argument("unknown cluster topology " + std::to_string(p.topology));
}

inline size_t n_constraints(const Platform& plat, const Params& p) {
  return plat.links.size() + (p.model == L07 ? size_t(plat.n_hosts) : 0);
}

// The network model's factors (network_cm02.cpp:36-64): LV08 = latency factor 13.01, bandwidth factor 0.97,
// weight_S 20537; CM02 = 1, 1, 0.
struct NetFactors {
  double latency, bandwidth, weight_s;
};
inline NetFactors net_factors(int model) {
  if (model == LV08)
    return {13.01, 0.97, 20537.0};
  if (model == CM02)
    return {1.0, 1.0, 0.0};
  throw std::invalid_argument("not a CM02-family network model: " + std::to_string(model));
}

// A link's constraint (NetworkCm02Link, network_cm02.cpp:282-295): bound = bandwidth factor * bandwidth,
// FATPIPE unshared.
template <class B>
typename B::Cnst link_constraint(B& b, int model, double bw, bool fatpipe) {
  typename B::Cnst c = b.constraint_new(net_factors(model).bandwidth * bw);
  if (fatpipe)
    b.unshare(c);
  return c;
}

// A WIFI access point's constraint (NetworkWifiLink, network_cm02.cpp:383-392): a shared link of bandwidth
// 1 / bandwidth factor, so that its bound is bandwidth factor * (1 / bandwidth factor) — 1 up to that rounding;
// a station's flow then takes 1 / rate of it per unit of rate (communicate).
template <class B>
typename B::Cnst wifi_link_constraint(B& b, int model) {
  const double bf = net_factors(model).bandwidth;
  return b.constraint_new(bf * (1.0 / bf));
}

// One communication, NetworkCm02Model::communicate (network_cm02.cpp:165-274): the action's latency (after the
// latency factor), its sharing penalty (the route latency + weight_S / bw per route link, in route order), the
// bound (rate < 0: TCP-gamma / (2 * route latency); else min(rate, that)), the variable — penalty 0 while the
// latency is unpaid (1 without latency), or, `paid`, the state once it is paid (update_actions_state restores
// the sharing penalty: network_cm02.cpp:105-146) — and its elements: each route link at 1.0, with
// crosstraffic each back-route link at 0.05.  route / back: indices into `links` and `cn`.  A WIFI route link
// (network_cm02.cpp:239-260) weighs 1 / the source station's rate, or the destination's when the source is not
// associated with that access point (neither associated: error); its bandwidth in the weight_S sum is the link's own,
// 1 / bandwidth factor (LinkImpl::get_bandwidth of the NetworkWifiLink).  WIFI with network/crosstraffic on (the
// `crosstraffic` flag, whether or not the back route has links) is the reference's assertion "Cross-traffic is not
// yet supported when using WIFI" (network_cm02.cpp:242): an error here too.
struct Comm {
  double latency;          // NetworkAction::latency_ (route latency * latency factor)
  double lat_current;      // lat_current_ (route latency)
  double sharing_penalty;  // sharing_penalty_
  double bound;            // the variable's bound
};
template <class B>
typename B::Var communicate(B& b, int model, const std::vector<Link>& links, const std::vector<typename B::Cnst>& cn,
                            const std::vector<int>& route, const std::vector<int>& back, double lat, double rate,
                            double tcp_gamma, bool paid, bool crosstraffic, Comm* out = nullptr) {
  const NetFactors f = net_factors(model);
  Comm a;
  a.sharing_penalty = lat;
  a.lat_current = lat;
  if (f.weight_s > 0)
    for (int l : route) {
      const Link& k = links[size_t(l)];
      a.sharing_penalty += f.weight_s / (k.wifi ? 1.0 / f.bandwidth : k.bw);
    }
  for (int l : route) {
    const Link& k = links[size_t(l)];
    if (!k.wifi)
      continue;
    if (crosstraffic)
      throw std::invalid_argument(
          "Cross-traffic is not yet supported when using WIFI. Please use --cfg=network/crosstraffic:0");
    if (k.src_rate == -1 && k.dst_rate == -1)
      throw std::invalid_argument("Some Stations are not associated to any Access Point. Make sure to call "
                                  "set_host_rate on all Stations.");
  }
  a.latency = lat * f.latency;
  if (rate < 0)
    a.bound = a.lat_current > 0 ? tcp_gamma / (2.0 * a.lat_current) : -1.0;
  else
    a.bound = a.lat_current > 0 ? std::min(rate, tcp_gamma / (2.0 * a.lat_current)) : rate;
  const double pen = a.latency > 0 ? (paid ? a.sharing_penalty : 0.0) : 1.0;
  typename B::Var v = b.variable_new(pen, a.bound, int(route.size() + back.size()));
  for (int l : route) {
    const Link& k = links[size_t(l)];
    // (src and dst on one access point: the source's rate, network_cm02.cpp:249-251)
    b.expand(cn[size_t(l)], v, !k.wifi ? 1.0 : k.src_rate != -1 ? 1.0 / k.src_rate : 1.0 / k.dst_rate);
  }
  for (int l : back)
    b.expand(cn[size_t(l)], v, 0.05);
  if (out)
    *out = a;
  return v;
}

// Links first (one constraint per link, network_cm02.cpp:286-295 / ptask_L07.cpp:247-255, FATPIPE
// unshared), then for L07 one CPU constraint per host (ptask_L07.cpp:239-240), then the flows.
template <class B>
void flows(B& b, const Platform& plat, const Params& p, std::vector<typename B::Cnst>* cnst_out,
           std::vector<typename B::Var>* var_out) {
  if (p.model < CM02 || p.model > L07)
    throw std::invalid_argument("unknown flow model " + std::to_string(p.model));
  if (plat.n_hosts <= 0)
    throw std::invalid_argument("platform without hosts");
  const bool l07 = p.model == L07;
  std::vector<typename B::Cnst> cn;
  cn.reserve(n_constraints(plat, p));
  for (const Link& l : plat.links) {
    if (l07) {
      cn.push_back(b.constraint_new(l.bw));
      if (l.fatpipe)
        b.unshare(cn.back());
    } else {
      cn.push_back(link_constraint(b, p.model, l.bw, l.fatpipe));
    }
  }
  const size_t cpu0 = cn.size();
  if (l07)
    for (int h = 0; h < plat.n_hosts; h++)
      cn.push_back(b.constraint_new(p.speed));

  lmm_gen::SplitMix64 r{p.seed * 0x9E3779B97F4A7C15ull + 7};
  std::vector<typename B::Var> vars;
  if (var_out)
    vars.reserve(size_t(p.n_flows));
  std::vector<int> route, back, uniq;
  for (int64_t f = 0; f < p.n_flows; f++) {
    const int src = int(r.next() % uint64_t(plat.n_hosts));
    const int dst = int(r.next() % uint64_t(plat.n_hosts));
    route.clear();
    double lat = 0.0;
    plat.route(src, dst, route, &lat);
    typename B::Var v;
    if (l07) {
      const double size = p.size_min + (p.size_max - p.size_min) * double(r.next() >> 11) * 0x1p-53;
      uniq = route;
      std::sort(uniq.begin(), uniq.end());
      uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
      // penalty 1 once the latency is paid, and the bound updateBound sets then (ptask_L07.cpp:389-417)
      const double bound = lat > 0 ? p.tcp_gamma / (2.0 * lat * size) : -1.0;
      v = b.variable_new(1.0, bound, int(2 + uniq.size()));
      b.expand(cn[cpu0 + size_t(src)], v, 0.0);
      b.expand(cn[cpu0 + size_t(dst)], v, 0.0);
      for (int l : route)
        b.expand_add(cn[size_t(l)], v, size);
    } else {
      back.clear();
      if (p.crosstraffic)
        plat.route(dst, src, back, nullptr);
      // rate -1 (no user rate), in the state once the latency is paid
      v = communicate(b, p.model, plat.links, cn, route, back, lat, -1.0, p.tcp_gamma, true, p.crosstraffic);
    }
    if (var_out)
      vars.push_back(v);
  }
  if (cnst_out)
    *cnst_out = std::move(cn);
  if (var_out)
    *var_out = std::move(vars);
}

}  // namespace lmm_plat
