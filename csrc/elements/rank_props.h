// Shared properties of the elements that talk to other ranks over a
// comm::Group (connect-type=RCCL edge / query elements, tensor_allgather).
#pragma once

#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "comm/group.h"
#include "core/util.h"
#include "runtime/element.h"
#include "runtime/hip_util.h"

namespace nnsx {

struct RankProps {
  int rank = -1;           // -1: $RANK
  int world = -1;          // -1: $WORLD_SIZE
  std::string ranks;       // "0,1,3": member global ranks ("" = all)
  std::string store;       // control-plane store host:port
  int backend = 0;         // auto | rccl | tcp
  unsigned timeout_ms = 0;  // 0: ini [rccl] timeout_ms (default 60000)
  int peer = -1;           // publisher / query server global rank (-1: first member)
  int device = -1;         // GPU of this member (-1: $LOCAL_RANK's GPU when any is visible)

  static const std::vector<std::string>& backends() {
    static const std::vector<std::string> b = {"auto", "rccl", "tcp"};
    return b;
  }

  // GPU this member's payloads live on (-1 = host only)
  int resolve_device() const {
    if (device >= 0) return device;
    if (backend == 2) return -1;
    const int n = hip::device_count();
    if (n <= 0) return -1;
    const char* lr = std::getenv("LOCAL_RANK");
    return (lr && *lr ? std::atoi(lr) : 0) % n;
  }

  // group rank of the peer (publisher / server) inside `g` (-1: not a member)
  int peer_in(const comm::Group& g) const {
    if (peer < 0) return 0;
    for (int i = 0; i < g.size(); ++i)
      if (g.global_rank(i) == peer) return i;
    return -1;
  }

  // register rank / world-size / group-ranks / peer-rank / device / store / comm-backend / comm-timeout
  // (with_device = false: the element owns a `device` property and copies it into `device`)
  void install(const std::function<PropSpec&(PropSpec)>& add, bool with_device = true) {
    auto num = [&](const char* n, int* t, const char* blurb) {
      PropSpec p;
      p.name = n;
      p.type = PropType::INT;
      p.blurb = blurb;
      p.set = [t](const std::string& v) { *t = std::stoi(v); };
      p.get = [t] { return std::to_string(*t); };
      add(p);
    };
    num("rank", &rank, "nnsx: global rank of this process (-1 = $RANK)");
    num("world-size", &world, "nnsx: number of ranks (-1 = $WORLD_SIZE)");
    num("peer-rank", &peer, "nnsx: global rank of the publisher / query server (-1 = first group member)");
    if (with_device)
      num("device", &device, "nnsx: GPU of this rank (-1 = $LOCAL_RANK's GPU when one is visible, else host)");
    PropSpec r;
    r.name = "group-ranks";
    r.blurb = "nnsx: comma-separated global ranks taking part (empty = all)";
    r.set = [this](const std::string& v) { ranks = v; };
    r.get = [this] { return ranks; };
    add(r);
    PropSpec st;
    st.name = "store";
    st.blurb = "nnsx: control-plane store host:port (empty = $NNSX_STORE or $MASTER_ADDR:$MASTER_PORT+17)";
    st.set = [this](const std::string& v) { store = v; };
    st.get = [this] { return store; };
    add(st);
    PropSpec b;
    b.name = "comm-backend";
    b.type = PropType::ENUM;
    b.choices = backends();
    b.blurb = "nnsx: data plane (auto = RCCL when every member has a GPU, else TCP through the store)";
    b.set = [this](const std::string& v) {
      for (size_t i = 0; i < backends().size(); ++i)
        if (backends()[i] == v || std::to_string(i) == v) backend = static_cast<int>(i);
    };
    b.get = [this] { return backends()[static_cast<size_t>(backend)]; };
    add(b);
    PropSpec t;
    t.name = "comm-timeout";
    t.type = PropType::UINT;
    t.blurb = "nnsx: rendezvous timeout (ms)";
    t.set = [this](const std::string& v) { timeout_ms = static_cast<unsigned>(std::stoul(v)); };
    t.get = [this] { return std::to_string(timeout_ms); };
    add(t);
  }

  comm::GroupSpec spec(const std::string& name) const {
    comm::GroupSpec s;
    s.name = name;
    s.rank = rank;
    s.world = world;
    s.device = resolve_device();
    for (auto& t : split(ranks, ',')) {
      const std::string v = strip(t);
      if (!v.empty()) s.members.push_back(std::stoi(v));
    }
    s.store = store;
    s.backend = backends()[static_cast<size_t>(backend)];
    s.timeout_ms = static_cast<int>(timeout_ms);
    return s;
  }

  // open (or reuse) the group; posts an element error on failure
  std::shared_ptr<comm::Group> open(Element* e, const std::string& name) const {
    std::string err;
    auto g = comm::group_get(spec(name), &err);
    if (!g) e->post_error(e->factory() + ": " + err);
    return g;
  }
};

}  // namespace nnsx
