// pin_registry.hpp -- host page-locking bookkeeping behind lsmgpu_host_register (api.hip).
//
// The reference's default loading mode is LoadToRAM (options.go:76): Table.mmap is then a Go heap
// buffer (table/table.go:117-123,329-338), neither page-aligned nor page-exclusive, and tables are
// opened and released all the time by compaction (levels.go:281-298), so pinned ranges share pages
// and address ranges come back.  Two facts of the HIP runtime shape this registry:
//  * pinning is page-granular, and a page must not be registered twice;
//  * a host copy is served from the registration its FIRST byte lies in, and one that runs past
//    that registration's end is rejected.
// So the library pins page-aligned, pairwise-disjoint SEGMENTS, each its own hipHostRegister, made
// of whole pages inside the callers' ranges (a range's partial first and last pages are never
// pinned: they may belong to other allocations).  A caller's range uses (references) every segment
// its pages overlap, and registering a range pins only the pages no segment covers yet.  Invariant: every pinned page lies in the pages of some
// live range.  When a range goes, a segment no live range overlaps is unpinned, and a segment
// other ranges still overlap only in part is RE-CUT (unpinned, its still-covered page runs pinned
// again): leaving it whole would keep pages of a freed buffer pinned, and a buffer mapped there
// later would be served from the stale pinned pages.  A re-cut unpins pages other ranges use, so
// the caller first drains the devices (api.hip holds the registry lock exclusively meanwhile,
// and every host copy is enqueued under the shared lock).  Every host copy the library issues is
// cut where segments begin and end (pieces()), so each piece lies inside one segment or outside
// all of them.
//
// Host-only C++ (no HIP types): tests/test_pin_registry.py compiles it into a CPU harness.
#pragma once
#include <algorithm>
#include <cstdint>
#include <iterator>
#include <map>
#include <shared_mutex>
#include <utility>
#include <vector>

namespace lsmgpu {

class PinRegistry {
 public:
  using Range = std::pair<uintptr_t, uintptr_t>;  // [first, second)

  explicit PinRegistry(uintptr_t page) : page_(page ? page : 4096) {}

  std::shared_mutex& mu() { return mu_; }
  uintptr_t page() const { return page_; }
  size_t segments() const { return segs_.size(); }
  size_t users() const { return uses_.size(); }

  // The whole pages inside [p, p + bytes) (possibly none).  Only those are pinned: the partial
  // first and last pages may hold other allocations' bytes (heap neighbours, the decode's own
  // output arrays allocated next to the input), and no copy into or out of such bytes may be
  // served through this registration's mapping -- round 5's GPU suite faulted (illegal memory
  // access in the pipeline's first device-to-host copy) with the ranges rounded OUT to pages.
  // The edge pieces (< 1 page each) are copied as pageable memory.
  Range page_range(uintptr_t p, uint64_t bytes) const {
    const uintptr_t a = (p + page_ - 1) / page_ * page_;
    const uintptr_t e = (p + bytes) / page_ * page_;
    return a < e ? Range{a, e} : Range{a, a};
  }

  // The page-aligned runs of [p, p + bytes)'s pages that no segment covers: what a register must
  // pin.  Caller holds mu().
  std::vector<Range> gaps(uintptr_t p, uint64_t bytes) const {
    const Range pr = page_range(p, bytes);
    std::vector<Range> out;
    if (pr.first >= pr.second) return out;
    uintptr_t cur = pr.first;
    auto it = first_overlapping(cur);
    while (cur < pr.second) {
      if (it == segs_.end() || it->first >= pr.second) {
        out.push_back({cur, pr.second});
        break;
      }
      if (it->first > cur) out.push_back({cur, it->first});
      cur = std::max(cur, it->second.e);
      ++it;
    }
    return out;
  }

  // Records a caller registration of [p, p + bytes): `made` are the gaps just pinned (they become
  // segments), then every segment overlapping the page range gains a user.  Caller holds mu().
  void add(uintptr_t p, uint64_t bytes, const std::vector<Range>& made) {
    for (const Range& m : made) segs_[m.first] = Seg{m.second, 0};
    const Range pr = page_range(p, bytes);
    if (pr.first < pr.second)  // (a range without a whole page uses no segment)
      for (auto it = first_overlapping(pr.first); it != segs_.end() && it->first < pr.second; ++it)
        it->second.refs++;
    uses_.emplace(p, pr);
  }

  // Drops the latest registration of pointer p.  False if p has none.  `unpin` receives the
  // segments to unpin (no live range overlaps them any more, or only in part), then `pin` the
  // page runs to pin again (the parts of re-cut segments live ranges still cover; they are
  // already segments here).  unpin_needs_drain: some unpinned segment is still in use by
  // another range (a re-cut), so in-flight copies must be drained first.  Caller holds mu().
  bool remove(uintptr_t p, std::vector<Range>* unpin, std::vector<Range>* pin,
              bool* unpin_needs_drain = nullptr) {
    if (unpin_needs_drain) *unpin_needs_drain = false;
    auto er = uses_.equal_range(p);
    if (er.first == er.second) return false;
    auto u = std::prev(er.second);  // equal keys keep insertion order: the latest
    const Range pr = u->second;
    uses_.erase(u);
    std::vector<Range> recut;
    for (auto it = pr.first < pr.second ? first_overlapping(pr.first) : segs_.end();
         it != segs_.end() && it->first < pr.second;) {
      const Range sg{it->first, it->second.e};
      if (--it->second.refs == 0) {
        unpin->push_back(sg);
        it = segs_.erase(it);
        continue;
      }
      // still used: keep it whole only if live ranges still cover every page of it
      std::vector<Range> cov = covered(sg);
      if (cov.size() == 1 && cov[0] == sg) {
        ++it;
        continue;
      }
      unpin->push_back(sg);
      if (unpin_needs_drain) *unpin_needs_drain = true;
      it = segs_.erase(it);
      for (const Range& c : cov) recut.push_back(c);
    }
    for (const Range& c : recut) {
      uint32_t refs = 0;
      for (const auto& kv : uses_)
        if (kv.second.first < c.second && c.first < kv.second.second) refs++;
      segs_[c.first] = Seg{c.second, refs};
      pin->push_back(c);
    }
    return true;
  }

  // Forgets a segment whose pinning failed (after a re-cut): its pages count as unpinned.
  void drop(const Range& r) {
    auto it = segs_.find(r.first);
    if (it != segs_.end() && it->second.e == r.second) segs_.erase(it);
  }

  // The host range [h, h + n) cut at segment borders: each piece lies inside one segment or
  // outside every segment.  Caller holds mu().
  void pieces(uintptr_t h, uint64_t n, std::vector<Range>* out) const {
    out->clear();
    const uintptr_t end = h + n;
    if (segs_.empty() || n == 0) {
      if (n) out->push_back({h, end});
      return;
    }
    uintptr_t cur = h;
    while (cur < end) {
      auto it = segs_.upper_bound(cur);  // first segment starting after cur
      uintptr_t stop = end;
      if (it != segs_.begin() && std::prev(it)->second.e > cur)
        stop = std::min(stop, std::prev(it)->second.e);  // inside that segment: to its end
      else if (it != segs_.end())
        stop = std::min(stop, it->first);  // outside: to the next segment's start
      out->push_back({cur, stop});
      cur = stop;
    }
  }

 private:
  struct Seg {
    uintptr_t e;    // segment = [key, e), page-aligned
    uint32_t refs;  // caller registrations whose pages overlap it
  };
  // the first segment that ends after `a` (segments are disjoint and sorted)
  std::map<uintptr_t, Seg>::const_iterator first_overlapping(uintptr_t a) const {
    auto it = segs_.upper_bound(a);
    if (it != segs_.begin() && std::prev(it)->second.e > a) return std::prev(it);
    return it;
  }
  std::map<uintptr_t, Seg>::iterator first_overlapping(uintptr_t a) {
    auto it = segs_.upper_bound(a);
    if (it != segs_.begin() && std::prev(it)->second.e > a) return std::prev(it);
    return it;
  }

  // the page runs of segment sg that live ranges cover (merged, sorted)
  std::vector<Range> covered(const Range& sg) const {
    std::vector<Range> iv;
    for (const auto& kv : uses_) {
      const uintptr_t a = std::max(kv.second.first, sg.first), e = std::min(kv.second.second, sg.second);
      if (a < e) iv.push_back({a, e});
    }
    std::sort(iv.begin(), iv.end());
    std::vector<Range> out;
    for (const Range& r : iv) {
      if (!out.empty() && r.first <= out.back().second)
        out.back().second = std::max(out.back().second, r.second);
      else
        out.push_back(r);
    }
    return out;
  }

  uintptr_t page_;
  std::map<uintptr_t, Seg> segs_;
  std::multimap<uintptr_t, Range> uses_;  // caller pointer -> its page range
  mutable std::shared_mutex mu_;
};

}  // namespace lsmgpu
