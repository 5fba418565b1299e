// CPU model check of lsmdb_amd/csrc/pin_registry.hpp (the bookkeeping behind
// lsmgpu_host_register): random register / unregister sequences over overlapping, page-sharing,
// nested, repeated and re-used ranges, against a page-level model of what HIP has pinned.
// Invariants checked after every step:
//   * no page is pinned twice (segments are disjoint; a gap never covers a pinned page);
//   * every page of every live range is pinned;
//   * a page is pinned only while some live range covers it (nothing leaks once all unregister);
//   * pieces() of any host range tile it exactly, and each piece lies inside one segment or
//     outside all of them.
// Built and run by tests/test_pin_registry.py: g++ -std=c++17 -O1 -I lsmdb_amd/csrc.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <set>
#include <vector>

#include "pin_registry.hpp"

using lsmgpu::PinRegistry;
using Range = PinRegistry::Range;

static int fails = 0;
#define CHECK(c, ...)                                \
  do {                                               \
    if (!(c)) {                                      \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                  \
      fprintf(stderr, "\n");                         \
      if (++fails > 20) exit(1);                     \
    }                                                \
  } while (0)

struct Model {
  uintptr_t page;
  std::map<uintptr_t, uintptr_t> pinned;  // segment start -> end, as "HIP" sees them
  std::map<uintptr_t, int> page_pins;     // page -> times pinned
  std::multimap<uintptr_t, uint64_t> live;  // caller pointer -> bytes

  void pin(Range r) {
    CHECK(r.first % page == 0 && r.second % page == 0 && r.first < r.second, "unaligned gap");
    CHECK(!pinned.count(r.first), "segment pinned twice at %lx", (unsigned long)r.first);
    pinned[r.first] = r.second;
    for (uintptr_t p = r.first; p < r.second; p += page) {
      CHECK(page_pins[p] == 0, "page %lx pinned twice", (unsigned long)p);
      page_pins[p]++;
    }
  }
  void unpin(Range r) {
    auto it = pinned.find(r.first);
    CHECK(it != pinned.end() && it->second == r.second, "unpin of a range never pinned");
    if (it != pinned.end()) pinned.erase(it);
    for (uintptr_t p = r.first; p < r.second; p += page) page_pins[p]--;
  }
  void check(const PinRegistry& R) {
    std::set<uintptr_t> need;
    for (auto& u : live) {
      Range pr = R.page_range(u.first, u.second);
      for (uintptr_t p = pr.first; p < pr.second; p += page) need.insert(p);
    }
    for (uintptr_t p : need) CHECK(page_pins[p] == 1, "live page %lx not pinned", (unsigned long)p);
    for (auto& kv : page_pins)
      if (kv.second) CHECK(need.count(kv.first), "page %lx pinned with no live range", (unsigned long)kv.first);
    CHECK(R.segments() == pinned.size(), "segment count %zu vs %zu", R.segments(), pinned.size());
  }
  // which pinned segment holds byte h (0 if none)
  uintptr_t seg_of(uintptr_t h) const {
    auto it = pinned.upper_bound(h);
    if (it == pinned.begin()) return 0;
    --it;
    return h < it->second ? it->first : 0;
  }
};

static void check_pieces(const PinRegistry& R, const Model& M, uintptr_t h, uint64_t n) {
  std::vector<Range> pc;
  R.pieces(h, n, &pc);
  uintptr_t cur = h;
  for (auto& r : pc) {
    CHECK(r.first == cur && r.second > r.first, "pieces do not tile the range");
    const uintptr_t s0 = M.seg_of(r.first), s1 = M.seg_of(r.second - 1);
    CHECK(s0 == s1, "piece [%lx,%lx) crosses a segment border", (unsigned long)r.first,
          (unsigned long)r.second);
    // a piece outside every segment must contain no pinned byte at all
    if (!s0) {
      auto it = M.pinned.lower_bound(r.first);
      CHECK(it == M.pinned.end() || it->first >= r.second, "unpinned piece covers a segment");
    }
    cur = r.second;
  }
  CHECK(cur == h + n, "pieces end at %lx, range at %lx", (unsigned long)cur, (unsigned long)(h + n));
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 20000;
  const uintptr_t page = 4096, base = 0x10000000;
  PinRegistry R(page);
  Model M{page, {}, {}, {}};
  std::mt19937_64 rng(12345);
  auto rnd = [&](uint64_t n) { return n ? rng() % n : 0; };

  // fixed scenarios first: the cases VERDICT r4 names
  {
    // two non-page-aligned buffers sharing a page
    std::vector<Range> g1 = R.gaps(base + 100, 5000), g2;
    for (auto& g : g1) M.pin(g);
    R.add(base + 100, 5000, g1);
    M.live.emplace(base + 100, 5000);
    g2 = R.gaps(base + 5200, 9000);
    // inward rounding: [base+100, +5000) pins no whole page... [base+5200, +9000) pins pages 2-3
    CHECK(g1.empty(), "a range without a whole page pinned something");
    CHECK(g2.size() == 1 && g2[0].first == base + 2 * page && g2[0].second == base + 3 * page,
          "whole inner pages");
    for (auto& g : g2) M.pin(g);
    R.add(base + 5200, 9000, g2);
    M.live.emplace(base + 5200, 9000);
    M.check(R);
    check_pieces(R, M, base + 5200, 9000);
    // unregister the first: the shared page stays pinned for the second
    std::vector<Range> rel, rep;
    CHECK(R.remove(base + 100, &rel, &rep), "remove");
    for (auto& r : rel) M.unpin(r);
    for (auto& r : rep) M.pin(r);
    M.live.erase(M.live.find(base + 100));
    M.check(R);
    CHECK(!R.remove(base + 100, &rel, &rep), "double remove accepted");
    rel.clear();
    rep.clear();
    CHECK(R.remove(base + 5200, &rel, &rep), "remove 2");
    for (auto& r : rel) M.unpin(r);
    CHECK(rep.empty(), "re-pin with no live range");
    M.live.clear();
    M.check(R);
    CHECK(R.segments() == 0 && R.users() == 0, "leak after the shared-page case");
    // register / unregister / register again at the same address
    for (int k = 0; k < 3; k++) {
      std::vector<Range> g = R.gaps(base + 64, 4 * page);
      CHECK(g.size() == 1 && g[0].second - g[0].first == 3 * page, "re-register gap count");
      for (auto& x : g) M.pin(x);
      R.add(base + 64, 4 * page, g);
      M.live.emplace(base + 64, 4 * page);
      M.check(R);
      rel.clear();
      rep.clear();
      CHECK(R.remove(base + 64, &rel, &rep) && rep.empty(), "remove re-registered");
      for (auto& r : rel) M.unpin(r);
      M.live.clear();
      M.check(R);
    }
    // the same pointer twice (two tables over one buffer): two users, one pin
    std::vector<Range> g = R.gaps(base, page);
    for (auto& x : g) M.pin(x);
    R.add(base, page, g);
    g = R.gaps(base, page);
    CHECK(g.empty(), "second registration of a pinned range pins again");
    R.add(base, page, g);
    rel.clear();
    rep.clear();
    CHECK(R.remove(base, &rel, &rep) && rel.empty() && rep.empty(),
          "first unregister unpinned a shared segment");
    CHECK(R.remove(base, &rel, &rep) && rel.size() == 1, "last unregister did not unpin");
    for (auto& r : rel) M.unpin(r);
    M.check(R);
  }

  // random sequences (the model's final check also covers the "all unregistered" state)
  std::vector<std::pair<uintptr_t, uint64_t>> handles;
  int regs = 0, unregs = 0, recuts = 0;
  for (int s = 0; s < steps; s++) {
    if (handles.empty() || rnd(100) < 55) {
      const uintptr_t p = base + rnd(64 * page);
      const uint64_t n = 1 + rnd(rnd(3) == 0 ? 12 * page : page);
      std::vector<Range> g = R.gaps(p, n);
      for (auto& x : g) M.pin(x);
      R.add(p, n, g);
      M.live.emplace(p, n);
      handles.push_back({p, n});
      regs++;
    } else {
      const size_t k = rnd(handles.size());
      const uintptr_t p = handles[k].first;
      std::vector<Range> rel, rep;
      bool drain = false;
      CHECK(R.remove(p, &rel, &rep, &drain), "remove of a live pointer failed");
      for (auto& r : rel) M.unpin(r);
      for (auto& r : rep) M.pin(r);
      recuts += drain ? 1 : 0;
      // the registry drops the latest registration of p: drop one model entry of p, and the
      // matching handle (the byte counts may differ, but page coverage is what is checked)
      auto er = M.live.equal_range(p);
      auto last = er.first;
      for (auto it = er.first; it != er.second; ++it) last = it;
      const uint64_t nb = last->second;
      M.live.erase(last);
      for (size_t j = handles.size(); j-- > 0;)
        if (handles[j].first == p && handles[j].second == nb) {
          handles.erase(handles.begin() + j);
          break;
        }
      unregs++;
    }
    M.check(R);
    const uintptr_t h = base + rnd(70 * page);
    check_pieces(R, M, h, 1 + rnd(16 * page));
  }
  while (!handles.empty()) {
    std::vector<Range> rel, rep;
    CHECK(R.remove(handles.back().first, &rel, &rep), "final remove");
    for (auto& r : rel) M.unpin(r);
    for (auto& r : rep) M.pin(r);
    handles.pop_back();
  }
  M.live.clear();
  M.check(R);
  CHECK(R.segments() == 0 && R.users() == 0, "registry not empty at the end");
  printf("{\"steps\": %d, \"registers\": %d, \"unregisters\": %d, \"recuts\": %d, \"fails\": %d}\n",
         steps, regs, unregs, recuts, fails);
  return fails ? 1 : 0;
}
