// api.hip -- the C ABI (include/lsmgpu.h) over the gfx950 codec kernels.
// Host-side responsibilities: argument validation, the SST tail parse (table.go:177-215),
// staging of host buffers through HBM, look-back scratch / epoch tags, block planning.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include <unistd.h>

#include "../../include/lsmgpu.h"
#include "kernels.hpp"
#include "host_io.hpp"

using namespace lsmgpu;

namespace {

constexpr uint32_t kTagMax = 0xfffffffeu;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t need) {
    if (need <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t n = std::max<size_t>(need, 256);
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

inline uint32_t rd_be32(const uint8_t* b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

// Ranges callers declared with lsmgpu_host_register (ABI 3 compatibility: bookkeeping only,
// nothing is page-locked -- host_io.hpp)
struct HostRanges {
  std::mutex mu;
  std::multimap<uintptr_t, uint64_t> r;
};
HostRanges& host_ranges() {
  static HostRanges h;
  return h;
}

// Synchronizes the given streams when the scope ends, on every return path: a call that returns
// (an error included) never leaves DMA into or out of the caller's host buffers in flight.
struct SyncOnExit {
  hipStream_t s[3] = {nullptr, nullptr, nullptr};
  ~SyncOnExit() {
    for (hipStream_t q : s)
      if (q) (void)hipStreamSynchronize(q);
  }
};

}  // namespace

struct lsmgpu_ctx {
  int device = 0;
  int num_cus = 256;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  DevBuf lb;             // look-back granules (64 B per block)
  DevBuf result;         // 8 x u64
  uint64_t* h_result = nullptr;  // pinned
  uint32_t tag = 0;
  DevBuf flags;          // encode flags
  DevBuf scan_tmp;
  DevBuf wsc;            // walk-scan-copy decode scratch (metadata, per-block triples)
  DevBuf open_tmp;       // batched table open: per-table scratch + scan temporary storage
  DevBuf merge_tmp;      // k-way merge: permutation, flags, tile bases, splitters
  // staging for host-memory calls
  DevBuf s_data, s_off, s_len, s_kd, s_ke, s_vd, s_ve, s_view, s_bf, s_bs, s_a, s_b, s_c, s_d;
  // kernel timing (lsmgpu_set_kernel_timing): events before the walk, between walk and copy,
  // after the copy of the last walk-scan-copy decode
  hipEvent_t kev[3] = {nullptr, nullptr, nullptr};
  bool ktime = false, kvalid = false, kfused = false;  // kfused: the last decode had no copy
  // lsmgpu_compact_tables: inputs, decoded / merged streams, cut arrays and the output images
  // (kept on the device until lsmgpu_compact_result copies them out)
  DevBuf cp_data, cp_off, cp_len, cp_kd, cp_ke, cp_vd, cp_ve, cp_bf, cp_bs, cp_res, cp_rf;
  DevBuf cp_msrc, cp_mke, cp_mve, cp_tf, cp_tb, cp_to, cp_out, cp_flags, cp_scratch;
  std::vector<uint64_t> cp_tbl_out;  // ntables + 1 image offsets of the last compaction
  uint64_t cp_bytes = 0;
  bool cp_valid = false;
  // host-memory decode pipeline (lsmgpu_decode_blocks, data_on_device = 0): copy-in / copy-out
  // streams, per-slot device buffers and events, pinned per-chunk result words
  static constexpr int kSlots = 3;
  hipStream_t s_in = nullptr, s_out = nullptr;
  struct Drain {  // a staged output piece: pin_out[at, at + n) -> caller dst, after out_done
    void* dst;
    uint64_t at, n;
  };
  struct Slot {
    DevBuf data, off, len, kd, ke, vd, ve, view, bf, bs, res;
    PinnedBuf pin_in, pin_out;  // staging of the chunk's input / outputs (pageable callers)
    std::vector<Drain> drains;  // outputs of the slot's chunk still to drain from pin_out
    bool in_used = false;       // in_done guards a DMA out of pin_in
    hipEvent_t in_done = nullptr, dec_done = nullptr, out_done = nullptr;
  } slot[kSlots];
  uint64_t* h_chunk_res = nullptr;  // pinned, 8 u64 per slot
  // every other host <-> HBM copy: direct DMA for runtime-pinned memory, else staged (host_io.hpp)
  CopyPool* pool = nullptr;
  Stager* stage = nullptr;
};

namespace {
inline hipError_t hcopy(lsmgpu_ctx* c, void* dst, const void* src, uint64_t n, hipMemcpyKind kind,
                        hipStream_t s) {
  return kind == hipMemcpyHostToDevice ? c->stage->h2d(dst, src, n, s) : c->stage->d2h(dst, src, n, s);
}
}  // namespace

// The failing HIP call and its error, kept per thread for lsmgpu_last_error; LSMGPU_DEBUG_ERR=1
// also prints it on stderr
static thread_local char t_last_error[256] = "";
static void report_hip_error(const char* what, hipError_t e, int line) {
  snprintf(t_last_error, sizeof(t_last_error), "%s -> %s (api.hip:%d)", what, hipGetErrorString(e), line);
  static const bool on = getenv("LSMGPU_DEBUG_ERR") != nullptr;
  if (on) fprintf(stderr, "lsmgpu: %s\n", t_last_error);
}
#define HIPC(x)                                    \
  do {                                             \
    hipError_t _e = (x);                           \
    if (_e != hipSuccess) {                        \
      report_hip_error(#x, _e, __LINE__);          \
      return LSMGPU_ERR_HIP;                       \
    }                                              \
  } while (0)

extern "C" {

int lsmgpu_abi_version(void) { return LSMGPU_ABI_VERSION; }

const char* lsmgpu_last_error(void) { return t_last_error; }

const char* lsmgpu_strerror(int code) {
  switch (code) {
    case LSMGPU_OK: return "ok";
    case LSMGPU_ERR_ARG: return "invalid argument";
    case LSMGPU_ERR_BAD_TAIL: return "malformed SST index tail";
    case LSMGPU_ERR_CAPACITY: return "output buffer too small";
    case LSMGPU_ERR_HIP: return "HIP runtime error";
    case LSMGPU_ERR_KEY_LEN: return "key length must be in (8, 65535]";
    case LSMGPU_ERR_VALUE_LEN: return "encoded value longer than 65535 bytes";
    case LSMGPU_ERR_TOO_LARGE: return "more than 4 GiB - 1 bytes in one call";
    case LSMGPU_ERR_INTERNAL: return "device look-back did not converge";
    case LSMGPU_ERR_NO_DEVICE: return "no HIP device";
    case LSMGPU_ERR_CORRUPT: return "corrupt input table (a block the iterator cannot walk)";
    case LSMGPU_ERR_HOST_PINNED: return "host memory already page-locked outside the library";
    default: return "unknown error";
  }
}

int lsmgpu_open(int device, lsmgpu_ctx** out) {
  if (!out) return LSMGPU_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LSMGPU_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return LSMGPU_ERR_NO_DEVICE;
  HIPC(hipSetDevice(device));
  lsmgpu_ctx* c = new lsmgpu_ctx();
  c->device = device;
  c->pool = new CopyPool(copy_threads());
  c->stage = new Stager(c->pool);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return LSMGPU_ERR_HIP;
  }
  c->stream = c->own_stream;
  if (c->result.ensure(64) != hipSuccess || c->flags.ensure(64) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_result), 64, hipHostMallocDefault) != hipSuccess) {
    lsmgpu_close(c);
    return LSMGPU_ERR_HIP;
  }
  *out = c;
  return LSMGPU_OK;
}

void lsmgpu_close(lsmgpu_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  // nothing may still run on the ctx's streams when their buffers and events go away
  for (hipStream_t q : {c->own_stream, c->stream, c->s_in, c->s_out})
    if (q) (void)hipStreamSynchronize(q);
  DevBuf* bufs[] = {&c->lb, &c->result, &c->flags, &c->scan_tmp, &c->wsc,
                    &c->open_tmp, &c->merge_tmp, &c->s_data,
                    &c->s_off, &c->s_len, &c->s_kd, &c->s_ke, &c->s_vd, &c->s_ve, &c->s_view,
                    &c->s_bf, &c->s_bs, &c->s_a, &c->s_b, &c->s_c, &c->s_d,
                    &c->cp_data, &c->cp_off, &c->cp_len, &c->cp_kd, &c->cp_ke, &c->cp_vd,
                    &c->cp_ve, &c->cp_bf, &c->cp_bs, &c->cp_res, &c->cp_rf, &c->cp_msrc,
                    &c->cp_mke, &c->cp_mve, &c->cp_tf, &c->cp_tb, &c->cp_to,
                    &c->cp_out, &c->cp_flags, &c->cp_scratch};
  for (DevBuf* b : bufs) b->release();
  if (c->stage) c->stage->release();
  delete c->stage;
  delete c->pool;
  for (auto& sl : c->slot) {
    DevBuf* sb[] = {&sl.data, &sl.off, &sl.len, &sl.kd, &sl.ke, &sl.vd, &sl.ve, &sl.view,
                    &sl.bf, &sl.bs, &sl.res};
    for (DevBuf* b : sb) b->release();
    sl.pin_in.release();
    sl.pin_out.release();
    for (hipEvent_t* e : {&sl.in_done, &sl.dec_done, &sl.out_done})
      if (*e) (void)hipEventDestroy(*e);
  }
  if (c->s_in) (void)hipStreamDestroy(c->s_in);
  if (c->s_out) (void)hipStreamDestroy(c->s_out);
  if (c->h_chunk_res) (void)hipHostFree(c->h_chunk_res);
  if (c->h_result) (void)hipHostFree(c->h_result);
  for (hipEvent_t& e : c->kev)
    if (e) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

int lsmgpu_set_stream(lsmgpu_ctx* c, void* s) {
  if (!c) return LSMGPU_ERR_ARG;
  c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
  return LSMGPU_OK;
}

void* lsmgpu_get_stream(lsmgpu_ctx* c) { return c ? reinterpret_cast<void*>(c->stream) : nullptr; }

int lsmgpu_synchronize(lsmgpu_ctx* c) {
  if (!c) return LSMGPU_ERR_ARG;
  HIPC(hipStreamSynchronize(c->stream));
  return LSMGPU_OK;
}

int lsmgpu_set_kernel_timing(lsmgpu_ctx* c, int on) {
  if (!c) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  if (on)
    for (hipEvent_t& e : c->kev)
      if (!e) HIPC(hipEventCreate(&e));
  c->ktime = on != 0;
  c->kvalid = false;
  return LSMGPU_OK;
}

int lsmgpu_kernel_times(lsmgpu_ctx* c, float* walk_ms, float* copy_ms) {
  if (!c || !walk_ms || !copy_ms) return LSMGPU_ERR_ARG;
  if (!c->kvalid) return LSMGPU_ERR_ARG;  // no timed walk-scan-copy decode yet
  HIPC(hipSetDevice(c->device));
  HIPC(hipEventSynchronize(c->kev[2]));
  HIPC(hipEventElapsedTime(walk_ms, c->kev[0], c->kev[1]));
  HIPC(hipEventElapsedTime(copy_ms, c->kev[1], c->kev[2]));
  if (c->kfused) *copy_ms = 0.0f;  // view-only decode finished in the walk: no copy launch
  return LSMGPU_OK;
}

int lsmgpu_stream_probe_async(lsmgpu_ctx* c, int kind, const void* d_src, void* d_dst,
                              uint64_t bytes, uint32_t wg_per_cu) {
  if (!c || !d_src || !d_dst || kind < 0 || kind > 7 || wg_per_cu == 0 || wg_per_cu > 64)
    return LSMGPU_ERR_ARG;
  // uint4 loads / stores: whole 16-B words at 16-B aligned addresses only
  if (bytes % 16 != 0 || ((uintptr_t)d_src | (uintptr_t)d_dst) % 16 != 0) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  HIPC(launch_stream_probe(kind, d_src, d_dst, bytes, wg_per_cu * (uint32_t)c->num_cus, c->stream));
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ index (table.go:177-215)
int lsmgpu_parse_index(const uint8_t* sst, uint64_t len, uint32_t* blk_off, uint32_t* blk_len,
                       uint64_t cap, uint64_t* nblk, uint64_t* bloom_off, uint64_t* bloom_len) {
  if (!sst || !nblk) return LSMGPU_ERR_ARG;
  *nblk = 0;
  if (len < 8) return LSMGPU_ERR_BAD_TAIL;
  uint64_t pos = len - 4;
  uint32_t bl = rd_be32(sst + pos);                    // table.go:181-183
  if (bl > pos || pos - bl < 4) return LSMGPU_ERR_BAD_TAIL;
  pos -= bl;
  if (bloom_off) *bloom_off = pos;
  if (bloom_len) *bloom_len = bl;
  pos -= 4;                                            // table.go:188-190
  uint32_t nr = rd_be32(sst + pos);
  if ((uint64_t)nr * 4 > pos) return LSMGPU_ERR_BAD_TAIL;
  pos -= (uint64_t)nr * 4;                             // table.go:192-199
  *nblk = nr;
  if (nr > cap || (nr && (!blk_off || !blk_len))) return LSMGPU_ERR_CAPACITY;
  uint32_t prev = 0;
  for (uint32_t i = 0; i < nr; i++) {                  // table.go:202-215
    uint32_t o = rd_be32(sst + pos + 4ull * i);
    if (o < prev || (uint64_t)o > pos) return LSMGPU_ERR_BAD_TAIL;
    blk_off[i] = prev;
    blk_len[i] = o - prev;
    prev = o;
  }
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ decode
static void next_tag(lsmgpu_ctx* c, uint64_t nblk) {
  if (c->tag >= kTagMax) {  // epoch wrap: clear every granule so stale tags cannot match
    (void)hipMemsetAsync(c->lb.p, 0, c->lb.cap, c->stream);
    c->tag = 0;
  }
  c->tag++;
  (void)nblk;
}

#ifdef LSMGPU_DIAG
}  // extern "C"
// The diagnostic build's A/B knobs over the rejected variants: LSMGPU_ABLATE,
// LSMGPU_WSC_{SPLIT,J,CHUNK,VIEWKEEP,TILE,ALIGN,LOOKBACK,BIDIR,PADLDS,TBE,PERSIST,EOSEP,EO,
// STAGECOPY,SUB,DPP,VIEWSCAN,SLOT} and LSMGPU_WSC_WALK=group2..group64
static void decode_diag_knobs(DecodeParams& p, uint64_t nblk, uint64_t cus, uint32_t max_blk_len,
                              const char* wk_env) {
  auto env = [](const char* n) { return getenv(n); };
  p.ablate = env("LSMGPU_ABLATE") ? (uint32_t)atoi(env("LSMGPU_ABLATE")) : 0u;
  if (const char* v = env("LSMGPU_WSC_SPLIT")) {
    const uint32_t sp = (uint32_t)atoi(v);
    p.wsplit = (sp == 2 || sp == 4) ? sp : 1u;
  }
  p.wj = env("LSMGPU_WSC_J") ? (uint32_t)atoi(env("LSMGPU_WSC_J")) : 0u;
  if (p.wj != 8 && p.wj != 16) p.wj = 0;
  if (const char* v = env("LSMGPU_WSC_CHUNK")) p.wchunk = atoi(v) == 16 ? 16u : 32u;
  if (const char* v = env("LSMGPU_WSC_VIEWKEEP")) p.wkeep = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_TILE")) {
    const int t = atoi(v);
    p.wtile = t == 192 || t == 128 || t == 64 ? (uint32_t)t : 256u;
  }
  p.walign = env("LSMGPU_WSC_ALIGN") ? (uint32_t)atoi(env("LSMGPU_WSC_ALIGN")) : 0u;
  if (const char* v = env("LSMGPU_WSC_LOOKBACK")) p.wlbfull = strcmp(v, "window") == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_BIDIR")) p.wbidir = (uint32_t)std::min(std::max(atoi(v), 0), 2);
  p.wpad = env("LSMGPU_WSC_PADLDS") ? (uint32_t)atoi(env("LSMGPU_WSC_PADLDS")) : 0u;
  if (p.wwide && env("LSMGPU_WSC_TBE") && atoi(env("LSMGPU_WSC_TBE")) == 0) p.wtbe = 576u;
  if (const char* v = env("LSMGPU_WSC_PERSIST")) p.wpersist = atoi(v) == 0 ? 0u : 1u;
  if (wk_env && strncmp(wk_env, "group", 5) == 0) {
    const int l = atoi(wk_env + 5);  // "group" alone: 8 lanes
    p.wlanes = l == 2 || l == 4 || l == 16 || l == 32 || l == 64 ? (uint32_t)l : 8u;
  }
  p.weosep = env("LSMGPU_WSC_EOSEP") && atoi(env("LSMGPU_WSC_EOSEP")) == 1 ? 1u : 0u;
  p.weo = p.wwalk == kWalkLane && !p.wfuse && env("LSMGPU_WSC_EO") && atoi(env("LSMGPU_WSC_EO")) == 1 ? 1u : 0u;
  const char* sc = env("LSMGPU_WSC_STAGECOPY");
  p.wscopy = p.wwalk == kWalkGroup && p.wlanes == 64 && !p.wfuse && !(sc && atoi(sc) == 0);
  p.wsub = env("LSMGPU_WSC_SUB") && atoi(env("LSMGPU_WSC_SUB")) == 1 ? 1u : 0u;
  p.wdpp = env("LSMGPU_WSC_DPP") && atoi(env("LSMGPU_WSC_DPP")) == 1 ? 1u : 0u;
  if (const char* v = env("LSMGPU_WSC_VIEWSCAN")) p.wview = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_DENSE")) p.wdense = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_PIPE")) p.wpipe = (uint32_t)std::min(std::max(atoi(v), 0), 2);  // 2: any n
  if (const char* v = env("LSMGPU_WSC_DPIPE")) p.wdpipe = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_DMAX")) p.wdmax = (uint32_t)atoi(v);
  if (const char* v = env("LSMGPU_WSC_DMIN")) p.wdmin = (uint32_t)atoi(v);
  if (const char* v = env("LSMGPU_WSC_LBIDIR")) p.wlbidir = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_B16")) p.wb16 = atoi(v) == 0 ? 0u : 1u;
  if (const char* v = env("LSMGPU_WSC_PDEPTH")) p.wpdepth = (uint32_t)std::min(std::max(atoi(v), 2), 4);
  const char* sl = env("LSMGPU_WSC_SLOT");
  p.wslot = sl && sl[0] == 's' ? 1u : (sl && sl[0] == 'n' ? 2u : 0u);
  (void)nblk;
  (void)cus;
  (void)max_blk_len;
}
extern "C" {
#endif

int lsmgpu_decode_blocks_async(lsmgpu_ctx* c, const uint8_t* d_data, uint64_t data_len,
                               const uint32_t* d_blk_off, const uint32_t* d_blk_len,
                               uint64_t nblk, uint32_t max_blk_len, int mode,
                               const lsmgpu_decoded* out, uint64_t* d_result) {
  if (!c || !out || !d_result) return LSMGPU_ERR_ARG;
  c->kvalid = false;  // kernel times describe this decode or none (other paths record none)
  if (mode & ~(LSMGPU_MODE_MATERIALIZE | LSMGPU_MODE_VIEW)) return LSMGPU_ERR_ARG;
  if (data_len > 0xffffffffull || nblk > 0xfffffffeull) return LSMGPU_ERR_TOO_LARGE;
  HIPC(hipSetDevice(c->device));
  if (nblk == 0) {
    HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
    if (out->blk_first) HIPC(hipMemsetAsync(out->blk_first, 0, 4, c->stream));
    return LSMGPU_OK;
  }
  if (!d_data || !d_blk_off || !d_blk_len) return LSMGPU_ERR_ARG;
  // layout: [gcnt: ngroups u32, padded to 256 B][block records 64 B x nblk][group records 64 B]
  const uint64_t ngroups = (nblk + 63) / 64;
  const size_t cnt_bytes = (size_t)((ngroups * 4 + 255) / 256 * 256);
  size_t need = cnt_bytes + (size_t)nblk * 64 + (size_t)ngroups * 64;
  if (need > c->lb.cap) {
    HIPC(hipStreamSynchronize(c->stream));
    HIPC(c->lb.ensure(need));
    HIPC(hipMemset(c->lb.p, 0, c->lb.cap));
  }
  next_tag(c, nblk);  // records are epoch-tagged: nothing to clear between launches
  DecodeParams p{};
  p.data = d_data;
  p.data_len = data_len;
  p.blk_off = d_blk_off;
  p.blk_len = d_blk_len;
  p.nblk = (uint32_t)nblk;
  p.mode = mode;
  p.key_data = out->key_data;
  p.key_cap = out->key_cap;
  p.key_end = out->key_end;
  p.val_data = out->val_data;
  p.val_cap = out->val_cap;
  p.val_end = out->val_end;
  p.view = out->view;
  p.ent_cap = out->ent_cap;
  p.blk_first = out->blk_first;
  p.blk_status = out->blk_status;
  p.gcnt = c->lb.as<uint32_t>();
  p.lb = reinterpret_cast<uint64_t*>(c->lb.as<uint8_t>() + cnt_bytes);
  p.glb = p.lb + nblk * 8;
  p.result = d_result;
  p.tag = c->tag;
  int path = decode_path(max_blk_len, (uint32_t)nblk);
  if (path == 2) {  // walk-scan-copy: blocks of 4 KiB .. 64 KiB - 1
    // entries of a block (>= 10 B each) + the sentinel, 4-B records rounded to 32-record
    // (128-B) chunks
    const uint32_t cap = (max_blk_len / 10 + 1 + 31) / 32 * 32;
    const size_t meta_b = (size_t)nblk * cap * 4;
    const size_t wneed = meta_b + (size_t)nblk * 32;  // records, then the 32-B descriptors
    if (wneed > c->wsc.cap) {
      HIPC(hipStreamSynchronize(c->stream));
      HIPC(c->wsc.ensure(wneed));
    }
    uint8_t* w = c->wsc.as<uint8_t>();
    p.wmeta = reinterpret_cast<uint32_t*>(w);
    p.wcap = cap;
    p.wdesc = reinterpret_cast<uint4*>(w + meta_b);  // (meta_b: 128-B chunks per block)
    const uint64_t cus = (uint64_t)c->num_cus;
    // The adopted configuration (DESIGN.md 5 has the measurements behind each choice):
    // * copy: two waves per block above 8 KiB (C5 1.25 -> 1.09 ms);
    // * view-only decodes finish inside the walk when there are >= 2 walk tiles (256 blocks) per
    //   CU (C2 1 GiB 0.413 -> 0.323 ms; with fewer the tile epilogues run on too few workgroups,
    //   C4 0.085 -> 0.165 ms);
    // * lane walks: 576-block tiles (9 waves, 2 workgroups per CU) when 256-block ones (4 per CU,
    //   LDS-bound) would not all be resident at once and 576-block ones would (C2 2^30 B: walk
    //   0.2296 -> 0.210 ms), sized for two equal waves of tiles (walk 0.2099 -> 0.2062 ms), and for
    //   materialize two tiles per workgroup walked back to back (walk 0.2059 -> 0.2011 ms);
    // * <= 64 blocks per CU (e.g. one 64 MiB table): 8 lanes per block guessing same-shape runs
    //   forward plus 8 walking backward from the terminator (C4 walk 0.0402 -> 0.0341 ms); else
    //   one lane per block (C2 1 GiB: lane 0.733 vs group 0.799 ms).
    // Test hooks (they choose among these compiled paths only): LSMGPU_WSC_VIEWFUSE=0|1,
    // LSMGPU_WSC_WIDE=0|1, LSMGPU_WSC_WALK=lane|group.
    p.wsplit = max_blk_len > 8192 ? 2u : 1u;
    const char* vf_env = getenv("LSMGPU_WSC_VIEWFUSE");
    const bool fuse = vf_env ? atoi(vf_env) != 0 : nblk >= 512ull * cus;
    p.wfuse = !(mode & LSMGPU_MODE_MATERIALIZE) && fuse;
    const char* ww_env = getenv("LSMGPU_WSC_WIDE");
    p.wwide = ww_env ? (atoi(ww_env) != 0 ? 576u : 0u)
                     : ((nblk + 255) / 256 > 4 * cus && (nblk + 575) / 576 <= 2 * cus ? 576u : 0u);
    p.wtbe = 576u;
    if (p.wwide) p.wtbe = (uint32_t)std::min<uint64_t>(576, std::max<uint64_t>(64, (nblk + 2 * cus - 1) / (2 * cus)));
    p.wwalk = nblk <= 64ull * cus ? kWalkGroup : kWalkLane;
    const char* wk_env = getenv("LSMGPU_WSC_WALK");
    if (wk_env && wk_env[0] == 'l') p.wwalk = kWalkLane;
    else if (wk_env && strncmp(wk_env, "group", 5) == 0) p.wwalk = kWalkGroup;
    p.wlanes = p.wwalk == kWalkGroup ? 8 : 1;
    // the diagnostic build's defaults of its extra knobs are the product's fixed choices
    p.wchunk = 32u;
    p.wkeep = 1u;
    // lane walks without wide tiles: 256-block tiles (128 / 64 when 256-block tiles would leave CUs
    // without one measured equal -- C5 walk 0.1831-0.1837 vs 0.1805-0.1824 ms, profiles/r06z --
    // so they stay in the diagnostic build, LSMGPU_WSC_TILE)
    p.wtile = 256u;
    p.wlbfull = 1u;
    p.wbidir = 1u;
    p.wpersist = 1u;
    p.wview = 1u;
    p.wdense = 1u;
    // the copy's pipelined 8-lane groups: every block of < 64 entries; blocks of >= 64 entries too
    // when the batch is large (100-entry blocks, compaction replay's 48 K: decode 0.403 -> 0.384
    // ms, profiles/r06w; one 64 MiB table, 5.4 K blocks of two waves each: copy 0.0307 -> 0.0335,
    // profiles/r06q)
    p.wpipe = nblk > 64ull * cus ? 2u : 1u;
    p.wdpipe = 1u;
    p.wdmax = 0xffffffffu;
    p.wdmin = 128u;
    p.wpdepth = 3u;
    // lane walks over blocks above 8 KiB: a second lane per block walks it backward
    p.wlbidir = max_blk_len > 8192 ? 1u : 0u;
    p.wb16 = 0u;
#ifdef LSMGPU_DIAG
    decode_diag_knobs(p, nblk, cus, max_blk_len, wk_env);
    // group walks: the copy in the walk's launch (LSMGPU_WSC_COPYFUSE=1), by workgroups past the
    // last walk ticket, each block copied once its tile is walked (only the 8 + 8 group walk)
    const char* cf_env = getenv("LSMGPU_WSC_COPYFUSE");
    p.wcopyfuse = p.wwalk == kWalkGroup && p.wlanes == 8 && p.wbidir == 1 && !p.wfuse &&
                  cf_env && atoi(cf_env) == 1 ? 1u : 0u;
    p.wncop = (uint32_t)std::min<uint64_t>((nblk + (p.wsplit == 1 ? 4 : 2) - 1) / (p.wsplit == 1 ? 4 : 2),
                                           6 * cus);  // (6 per CU: with the walk, ~7 resident)
#endif
    // d_result is zeroed by the walk kernel when a copy launch follows it (the copy's atomics
    // come after the kernel boundary): one operation fewer per decode.  A view-only decode
    // that ends in the walk updates d_result from every workgroup, so it is zeroed first.
#ifdef LSMGPU_STAMPS
    if (getenv("LSMGPU_STAMPS")) {  // diagnostic build: the walk's per-tile stamps (decode_wsc.hip)
      static DevBuf stamp_buf;
      HIPC(stamp_buf.ensure((16 + (size_t)nblk * 4) * 8));
      p.stamps = stamp_buf.as<uint64_t>();
      HIPC(hipMemsetAsync(p.stamps, 0, 16 * sizeof(uint64_t), c->stream));  // walk counters
    }
#endif
    if (p.wfuse || LSMGPU_KNOB(p.wscopy, 0u)) HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
    else p.zero_result = 1;
    if (c->ktime) HIPC(hipEventRecord(c->kev[0], c->stream));
    HIPC(launch_decode_wsc(p, c->stream, c->ktime ? c->kev[1] : nullptr));
    if (c->ktime) HIPC(hipEventRecord(c->kev[2], c->stream));
    c->kvalid = c->ktime;
    c->kfused = p.wfuse != 0 || LSMGPU_KNOB(p.wcopyfuse, 0u) != 0;
    return LSMGPU_OK;
  }
  uint64_t waves = 0;
  HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
  HIPC(launch_decode(p, max_blk_len, c->num_cus, c->stream, &waves));
  (void)waves;
  return LSMGPU_OK;
}

// ABI 4: no page-locking (host_io.hpp); the registry keeps ABI 3's argument and error rules
int lsmgpu_host_register(lsmgpu_ctx* c, void* p, uint64_t bytes) {
  if (!c || !p || !bytes || (uintptr_t)p + bytes < (uintptr_t)p) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  // page-locked outside this library (hipHostMalloc, lsmgpu_host_alloc, a caller's own
  // hipHostRegister): it is DMA'd directly and needs no registration
  const uint8_t* q = static_cast<const uint8_t*>(p);
  if (runtime_pinned(q, 1) || runtime_pinned(q + bytes - 1, 1)) return LSMGPU_ERR_HOST_PINNED;
  HostRanges& R = host_ranges();
  std::lock_guard<std::mutex> g(R.mu);
  R.r.emplace((uintptr_t)p, bytes);
  return LSMGPU_OK;
}

int lsmgpu_host_unregister(lsmgpu_ctx* c, void* p) {
  if (!c || !p) return LSMGPU_ERR_ARG;
  HostRanges& R = host_ranges();
  std::lock_guard<std::mutex> g(R.mu);
  auto it = R.r.find((uintptr_t)p);
  if (it == R.r.end()) return LSMGPU_ERR_ARG;  // not registered
  R.r.erase(it);
  return LSMGPU_OK;
}

int lsmgpu_host_alloc(lsmgpu_ctx* c, uint64_t bytes, void** out) {
  if (!c || !out || !bytes) return LSMGPU_ERR_ARG;
  *out = nullptr;
  HIPC(hipSetDevice(c->device));
  HIPC(hipHostMalloc(out, bytes, hipHostMallocPortable));
  return LSMGPU_OK;
}

int lsmgpu_host_free(lsmgpu_ctx* c, void* p) {
  if (!p) return LSMGPU_OK;
  if (c) HIPC(hipSetDevice(c->device));
  HIPC(hipHostFree(p));
  return LSMGPU_OK;
}

}  // extern "C"

namespace {

// key_end / val_end / blk_first of one chunk of a pipelined host decode += the entries, key
// bytes and value bytes of the chunks before it (the chunk was decoded with bases 0)
__global__ void __launch_bounds__(256) add_bases_kernel(uint32_t* ke, uint32_t* ve, uint32_t n,
                                                        uint32_t kb, uint32_t vb, uint32_t* bf,
                                                        uint32_t nb1, uint32_t eb) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (ke) ke[i] += kb;
    if (ve) ve[i] += vb;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb1; i += stride) bf[i] += eb;
}

constexpr int kNotPipelined = -1;

// A pipeline slot's staged outputs into the caller's arrays, once their D2H has landed
hipError_t drain(lsmgpu_ctx* c, lsmgpu_ctx::Slot& sl) {
  if (sl.drains.empty()) return hipSuccess;
  const hipError_t e = hipEventSynchronize(sl.out_done);
  if (e != hipSuccess) return e;
  for (const auto& d : sl.drains) c->pool->copy(d.dst, sl.pin_out.p + d.at, d.n);
  sl.drains.clear();
  return hipSuccess;
}

// lsmgpu_decode_blocks for host memory, as a pipeline: the blocks (sorted by offset, disjoint)
// are cut into chunks of ~64 MiB of input; chunk c's copy-in (s_in), decode (ctx stream) and
// copy-out (s_out) overlap chunk c+1's copy-in and chunk c-1's copy-out, over kSlots device
// slots.  Each chunk decodes with bases 0; once its decode has finished the host knows the
// chunk's totals, adds the bases of the chunks before it on the device (add_bases_kernel) and
// copies the outputs to their places.  Returns kNotPipelined when the batch is one chunk, the
// blocks are unsorted or a chunk overflows its device slot (prefix-compressed keys that expand):
// the caller then decodes in one shot.
int decode_host_pipelined(lsmgpu_ctx* c, const uint8_t* data, uint64_t data_len,
                          const uint32_t* blk_off, const uint32_t* blk_len, uint64_t nblk,
                          int mode, lsmgpu_decoded* out, uint32_t max_len) {
  const char* ch_env = getenv("LSMGPU_HOST_CHUNK");
  const uint64_t chunk = ch_env && atoll(ch_env) >= (1 << 20) ? (uint64_t)atoll(ch_env) : (32ull << 20);
  if (max_len >= 65536 || nblk < 2) return kNotPipelined;
  for (uint64_t b = 0; b < nblk; b++) {
    if ((uint64_t)blk_off[b] + blk_len[b] > data_len) return kNotPipelined;
    if (b && blk_off[b] < (uint64_t)blk_off[b - 1] + blk_len[b - 1]) return kNotPipelined;
  }
  std::vector<uint64_t> cb{0};  // chunk c = blocks [cb[c], cb[c+1])
  for (uint64_t b = 1; b < nblk; b++)
    if ((uint64_t)blk_off[b] + blk_len[b] - blk_off[cb.back()] > chunk) cb.push_back(b);
  cb.push_back(nblk);
  const uint64_t nch = cb.size() - 1;
  if (nch < 2) return kNotPipelined;
  uint64_t max_span = 0, max_nb = 0;
  for (uint64_t k = 0; k < nch; k++) {
    const uint64_t a = blk_off[cb[k]] & ~127ull, e = (uint64_t)blk_off[cb[k + 1] - 1] + blk_len[cb[k + 1] - 1];
    max_span = std::max(max_span, e - a);
    max_nb = std::max(max_nb, cb[k + 1] - cb[k]);
  }
  const bool mat = (mode & LSMGPU_MODE_MATERIALIZE) != 0, view = (mode & LSMGPU_MODE_VIEW) != 0;
  const uint64_t ecap = max_span / 10 + 1;  // >= 10 B per entry (its header)
  // input: DMA'd straight from runtime-pinned memory (lsmgpu_host_alloc), else memcpy'd into the
  // slot's pin_in first; the chunk's block offsets / lengths always go through pin_in
  const bool in_direct = runtime_pinned(data, data_len);
  const uint64_t idx_at_max = in_direct ? 0 : (max_span + 255) / 256 * 256;
  if (!c->s_in) HIPC(hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking));
  if (!c->s_out) HIPC(hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
  if (!c->h_chunk_res)
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->h_chunk_res), 64 * lsmgpu_ctx::kSlots,
                       hipHostMallocDefault));
  for (auto& sl : c->slot) {
    HIPC(sl.data.ensure(max_span + 256));
    HIPC(sl.off.ensure(max_nb * 4 + 4));
    HIPC(sl.len.ensure(max_nb * 4 + 4));
    HIPC(sl.bf.ensure(max_nb * 4 + 8));
    HIPC(sl.bs.ensure(max_nb * 4 + 4));
    HIPC(sl.res.ensure(64));
    if (mat) {
      HIPC(sl.kd.ensure(max_span + 16));
      HIPC(sl.vd.ensure(max_span + 16));
      HIPC(sl.ke.ensure(ecap * 4));
      HIPC(sl.ve.ensure(ecap * 4));
    }
    if (view) HIPC(sl.view.ensure(ecap * 8));
    for (hipEvent_t* e : {&sl.in_done, &sl.dec_done, &sl.out_done})
      if (!*e) HIPC(hipEventCreateWithFlags(e, hipEventDisableTiming));
    // (no DMA of an earlier call is in flight: every call drains its streams before returning)
    HIPC(sl.pin_in.ensure(idx_at_max + max_nb * 8 + 256));
    sl.drains.clear();
    sl.in_used = false;
  }
  // every return below (errors included) first drains the three streams: no copy into the
  // caller's arrays outlives the call
  SyncOnExit drain_all;
  drain_all.s[0] = c->s_in;
  drain_all.s[1] = c->stream;
  drain_all.s[2] = c->s_out;
  // running totals of the chunks already placed
  uint64_t E = 0, KB = 0, VB = 0, nbad = 0;
  int64_t first_bad = -1;
  bool fits = true;
  std::vector<uint8_t> slot_used(lsmgpu_ctx::kSlots, 0);
  for (uint64_t i = 0; i <= nch; i++) {
    if (i < nch) {  // chunk i: copy in, decode
      auto& sl = c->slot[i % lsmgpu_ctx::kSlots];
      const uint64_t b0 = cb[i], nb = cb[i + 1] - b0;
      const uint64_t a = blk_off[b0] & ~127ull, e = (uint64_t)blk_off[cb[i + 1] - 1] + blk_len[cb[i + 1] - 1];
      if (sl.in_used) HIPC(hipEventSynchronize(sl.in_done));  // pin_in's last DMA is done
      const uint64_t idx_at = in_direct ? 0 : (e - a + 255) / 256 * 256;
      const uint8_t* src = data + a;
      if (!in_direct) {
        c->pool->copy(sl.pin_in.p, data + a, e - a);
        src = sl.pin_in.p;
      }
      std::memcpy(sl.pin_in.p + idx_at, blk_off + b0, nb * 4);
      std::memcpy(sl.pin_in.p + idx_at + nb * 4, blk_len + b0, nb * 4);
      if (slot_used[i % lsmgpu_ctx::kSlots]) HIPC(hipStreamWaitEvent(c->s_in, sl.out_done, 0));
      slot_used[i % lsmgpu_ctx::kSlots] = 1;
      HIPC(hipMemcpyAsync(sl.data.p, src, e - a, hipMemcpyHostToDevice, c->s_in));
      HIPC(hipMemcpyAsync(sl.off.p, sl.pin_in.p + idx_at, nb * 4, hipMemcpyHostToDevice, c->s_in));
      HIPC(hipMemcpyAsync(sl.len.p, sl.pin_in.p + idx_at + nb * 4, nb * 4, hipMemcpyHostToDevice,
                          c->s_in));
      HIPC(hipEventRecord(sl.in_done, c->s_in));
      sl.in_used = true;
      HIPC(hipStreamWaitEvent(c->stream, sl.in_done, 0));
      lsmgpu_decoded d{};
      if (mat) {
        d.key_data = sl.kd.as<uint8_t>();
        d.key_cap = max_span;
        d.key_end = sl.ke.as<uint32_t>();
        d.val_data = sl.vd.as<uint8_t>();
        d.val_cap = max_span;
        d.val_end = sl.ve.as<uint32_t>();
      }
      if (view) d.view = sl.view.as<uint64_t>();
      d.ent_cap = ecap;
      d.blk_first = sl.bf.as<uint32_t>();
      d.blk_status = sl.bs.as<int32_t>();
      uint32_t ml = 0;
      for (uint64_t b = b0; b < b0 + nb; b++) ml = std::max(ml, blk_len[b]);
      // the slot holds data[a, e): the kernels see it through a pointer biased by -a, so the
      // caller's offsets (and the view records' key positions) stay absolute
      int rc = lsmgpu_decode_blocks_async(c, sl.data.as<uint8_t>() - a, e,
                                          sl.off.as<uint32_t>(), sl.len.as<uint32_t>(), nb, ml,
                                          mode, &d, sl.res.as<uint64_t>());
      if (rc != LSMGPU_OK) return rc;
      HIPC(hipMemcpyAsync(c->h_chunk_res + 8 * (i % lsmgpu_ctx::kSlots), sl.res.p, 64,
                          hipMemcpyDeviceToHost, c->stream));
      HIPC(hipEventRecord(sl.dec_done, c->stream));
    }
    if (i == 0) continue;
    // chunk j = i - 1: its totals, then the bases and the copy-out
    const uint64_t j = i - 1, b0 = cb[j], nb = cb[j + 1] - b0;
    auto& sl = c->slot[j % lsmgpu_ctx::kSlots];
    HIPC(hipEventSynchronize(sl.dec_done));
    const uint64_t* r = c->h_chunk_res + 8 * (j % lsmgpu_ctx::kSlots);
    const uint64_t n = r[0], kb = r[1], vb = r[2], fb = r[3], bad = r[4], fl = r[5];
    if (fl & 2) return LSMGPU_ERR_INTERNAL;
    if (fl & 1) return kNotPipelined;  // a chunk outgrew its slot (expanding prefix-compressed keys)
    if (fb && first_bad < 0) first_bad = (int64_t)(b0 + nb - fb);
    nbad += bad;
    fits = fits && E + n <= out->ent_cap && E + n <= 0xffffffffull &&
           (!out->key_data || KB + kb <= out->key_cap) && (!out->val_data || VB + vb <= out->val_cap) &&
           KB + kb < 0xffffffffull && VB + vb <= 0xffffffffull;
    HIPC(hipStreamWaitEvent(c->s_out, sl.dec_done, 0));
    const bool last = j + 1 == nch;
    if (E | KB | VB) {
      const uint32_t nb1 = (uint32_t)nb + (last ? 1 : 0);
      hipLaunchKernelGGL(add_bases_kernel, dim3(512), dim3(256), 0, c->s_out,
                         mat && fits && out->key_end ? sl.ke.as<uint32_t>() : nullptr,
                         mat && fits && out->val_end ? sl.ve.as<uint32_t>() : nullptr,
                         fits ? (uint32_t)n : 0u, (uint32_t)KB, (uint32_t)VB, sl.bf.as<uint32_t>(),
                         out->blk_first ? nb1 : 0u, (uint32_t)E);
      HIPC(hipGetLastError());
    }
    // outputs: straight into runtime-pinned caller arrays, else into the slot's pin_out, drained
    // into the caller's arrays by the host while the next chunk's copies run
    struct Piece {
      void* hp;
      const void* dp;
      uint64_t n;
    } pcs[7];
    int np = 0;
    auto add = [&](void* hp, const void* dp, uint64_t bytes) {
      if (hp && bytes) pcs[np++] = {hp, dp, bytes};
    };
    if (fits) {
      if (mat) {
        add(out->key_data ? out->key_data + KB : nullptr, sl.kd.p, kb);
        add(out->val_data ? out->val_data + VB : nullptr, sl.vd.p, vb);
        add(out->key_end ? out->key_end + E : nullptr, sl.ke.p, n * 4);
        add(out->val_end ? out->val_end + E : nullptr, sl.ve.p, n * 4);
      }
      if (view) add(out->view ? out->view + E : nullptr, sl.view.p, n * 8);
    }
    add(out->blk_first ? out->blk_first + b0 : nullptr, sl.bf.p, (nb + (last ? 1 : 0)) * 4);
    add(out->blk_status ? out->blk_status + b0 : nullptr, sl.bs.p, nb * 4);
    bool direct[7];
    uint64_t need = 0;
    for (int k = 0; k < np; k++) {
      direct[k] = runtime_pinned(pcs[k].hp, pcs[k].n);
      if (!direct[k]) need += (pcs[k].n + 15) / 16 * 16;
    }
    // (slot j's previous chunk, j - kSlots, was drained while chunk j - 1 was placed)
    HIPC(sl.pin_out.ensure(need));
    uint64_t at = 0;
    for (int k = 0; k < np; k++) {
      if (direct[k]) {
        HIPC(hipMemcpyAsync(pcs[k].hp, pcs[k].dp, pcs[k].n, hipMemcpyDeviceToHost, c->s_out));
      } else {
        HIPC(hipMemcpyAsync(sl.pin_out.p + at, pcs[k].dp, pcs[k].n, hipMemcpyDeviceToHost, c->s_out));
        sl.drains.push_back({pcs[k].hp, at, pcs[k].n});
        at += (pcs[k].n + 15) / 16 * 16;
      }
    }
    HIPC(hipEventRecord(sl.out_done, c->s_out));
    if (j) HIPC(drain(c, c->slot[(j - 1) % lsmgpu_ctx::kSlots]));
    E += n;
    KB += kb;
    VB += vb;
  }
  HIPC(drain(c, c->slot[(nch - 1) % lsmgpu_ctx::kSlots]));
  HIPC(hipStreamSynchronize(c->s_out));
  out->n_entries = E;
  out->key_bytes = KB;
  out->val_bytes = VB;
  out->first_bad_block = first_bad;
  out->n_bad_blocks = nbad;
  return fits ? LSMGPU_OK : LSMGPU_ERR_CAPACITY;
}

}  // namespace

extern "C" {

int lsmgpu_decode_blocks(lsmgpu_ctx* c, const uint8_t* data, uint64_t data_len,
                         int data_on_device, const uint32_t* blk_off, const uint32_t* blk_len,
                         uint64_t nblk, int mode, lsmgpu_decoded* out) {
  if (!c || !out) return LSMGPU_ERR_ARG;
  if (nblk && (!blk_off || !blk_len || !data)) return LSMGPU_ERR_ARG;
  if (data_len > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  if (mode & ~(LSMGPU_MODE_MATERIALIZE | LSMGPU_MODE_VIEW)) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  if (!data_on_device && data_len && device_memory(data)) return LSMGPU_ERR_ARG;  // (flag mismatch)
  uint32_t max_len = 0;
  for (uint64_t b = 0; b < nblk; b++) max_len = std::max(max_len, blk_len[b]);
  const bool query0 = !out->key_data && !out->key_end && !out->val_data && !out->val_end &&
                      !out->view && !out->blk_first && !out->blk_status;
  if (!data_on_device && !query0) {  // host memory: the chunked copy-in / decode / copy-out pipeline
    const int prc = decode_host_pipelined(c, data, data_len, blk_off, blk_len, nblk, mode, out, max_len);
    if (prc != kNotPipelined) return prc;
  }
  SyncOnExit sync_exit;  // no DMA into the caller's arrays outlives the call, errors included
  sync_exit.s[0] = c->stream;
  HIPC(c->s_off.ensure((nblk + 1) * 4));
  HIPC(c->s_len.ensure((nblk + 1) * 4));
  if (nblk) {
    HIPC(hcopy(c, c->s_off.p, blk_off, nblk * 4, hipMemcpyHostToDevice, c->stream));
    HIPC(hcopy(c, c->s_len.p, blk_len, nblk * 4, hipMemcpyHostToDevice, c->stream));
  }
  lsmgpu_decoded d = *out;
  // every output pointer NULL = a size query: the blocks are walked, n_entries / key_bytes /
  // val_bytes / first_bad_block / n_bad_blocks report what a materialize (or view) call needs
  const bool query = !out->key_data && !out->key_end && !out->val_data && !out->val_end &&
                     !out->view && !out->blk_first && !out->blk_status;
  if (query) {
    d.key_cap = d.val_cap = d.ent_cap = ~0ull;
    mode = LSMGPU_MODE_VIEW;
  }
  const uint8_t* d_data = data;
  if (!data_on_device) {  // stage host buffers through HBM
    HIPC(c->s_data.ensure(data_len + 16));
    if (data_len) HIPC(hcopy(c, c->s_data.p, data, data_len, hipMemcpyHostToDevice, c->stream));
    d_data = c->s_data.as<uint8_t>();
    auto stage = [&](DevBuf& b, void* hp, uint64_t bytes) -> void* {
      if (!hp) return nullptr;
      if (b.ensure(bytes + 16) != hipSuccess) return (void*)-1;
      return b.p;
    };
    d.key_data = (uint8_t*)stage(c->s_kd, out->key_data, out->key_cap);
    d.val_data = (uint8_t*)stage(c->s_vd, out->val_data, out->val_cap);
    d.key_end = (uint32_t*)stage(c->s_ke, out->key_end, out->ent_cap * 4);
    d.val_end = (uint32_t*)stage(c->s_ve, out->val_end, out->ent_cap * 4);
    d.view = (uint64_t*)stage(c->s_view, out->view, out->ent_cap * 8);
    d.blk_first = (uint32_t*)stage(c->s_bf, out->blk_first, (nblk + 1) * 4);
    d.blk_status = (int32_t*)stage(c->s_bs, out->blk_status, nblk * 4);
    void* ptrs[] = {d.key_data, d.val_data, d.key_end, d.val_end, d.view, d.blk_first, d.blk_status};
    for (void* q : ptrs)
      if (q == (void*)-1) return LSMGPU_ERR_HIP;
  }
  int rc = lsmgpu_decode_blocks_async(c, d_data, data_len, c->s_off.as<uint32_t>(),
                                      c->s_len.as<uint32_t>(), nblk, max_len, mode, &d,
                                      c->result.as<uint64_t>());
  if (rc != LSMGPU_OK) return rc;
  HIPC(hipMemcpyAsync(c->h_result, c->result.p, 64, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  const uint64_t* r = c->h_result;
  out->n_entries = r[0];
  out->key_bytes = r[1];
  out->val_bytes = r[2];
  out->first_bad_block = r[3] ? (int64_t)(nblk - r[3]) : -1;
  out->n_bad_blocks = r[4];
  const uint64_t flags = r[5];
  if (!data_on_device) {
    auto back = [&](void* hp, const void* dp, uint64_t bytes) -> hipError_t {
      if (!hp || !bytes) return hipSuccess;
      return hcopy(c, hp, dp, bytes, hipMemcpyDeviceToHost, c->stream);
    };
    const bool fits = !(flags & 1);
    uint64_t ne = fits ? out->n_entries : 0;
    if (fits) {
      HIPC(back(out->key_data, d.key_data, std::min(out->key_cap, out->key_bytes)));
      HIPC(back(out->val_data, d.val_data, std::min(out->val_cap, out->val_bytes)));
      HIPC(back(out->key_end, d.key_end, ne * 4));
      HIPC(back(out->val_end, d.val_end, ne * 4));
      HIPC(back(out->view, d.view, ne * 8));
    }
    HIPC(back(out->blk_first, d.blk_first, (nblk + 1) * 4));
    HIPC(back(out->blk_status, d.blk_status, nblk * 4));
    HIPC(hipStreamSynchronize(c->stream));
  }
  if (flags & 2) return LSMGPU_ERR_INTERNAL;
  if (flags & 1) return LSMGPU_ERR_CAPACITY;
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ encode
int lsmgpu_plan_blocks(const uint32_t* key_end, const uint32_t* vs_end, uint64_t n,
                       uint32_t epb, uint32_t block_bytes, uint32_t* blk_first, uint64_t cap,
                       uint64_t* nblocks) {
  if (!nblocks || (n && (!key_end || !vs_end))) return LSMGPU_ERR_ARG;
  if (epb == 0 && block_bytes == 0) return LSMGPU_ERR_ARG;
  // Builder.Add (builder.go:125-137) cut rule, plus the opt-in byte target
  uint64_t nb = 0, counter = 0, cur = 0;
  auto emit = [&](uint64_t e) {
    if (blk_first && nb < cap) blk_first[nb] = (uint32_t)e;
    nb++;
  };
  emit(0);
  uint32_t k0 = 0, v0 = 0;
  for (uint64_t e = 0; e < n; e++) {
    uint64_t sz = 10ull + (key_end[e] - k0) + (vs_end[e] - v0);
    k0 = key_end[e];
    v0 = vs_end[e];
    bool cut = (epb > 0 && counter >= epb);
    if (!cut && block_bytes > 0 && counter > 0) cut = (cur + sz + 13) > block_bytes;
    if (cut) {
      emit(e);
      counter = 0;
      cur = 0;
    }
    counter++;
    cur += sz;
  }
  if (blk_first && nb < cap) blk_first[nb] = (uint32_t)n;  // end sentinel
  *nblocks = nb;
  return (nb + 1 <= cap || !blk_first) ? LSMGPU_OK : LSMGPU_ERR_CAPACITY;
}

int lsmgpu_encode_blocks_async(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                               const uint8_t* d_vs, const uint32_t* d_vs_end, uint64_t n,
                               uint32_t epb, const uint32_t* d_blk_first, uint64_t nblocks,
                               uint64_t key_total, uint64_t vs_total, uint8_t* d_out,
                               uint64_t out_cap, uint32_t* d_flags) {
  if (!c || !d_out || !d_flags) return LSMGPU_ERR_ARG;
  if (n && (!d_keys || !d_key_end || !d_vs || !d_vs_end)) return LSMGPU_ERR_ARG;
  if (!d_blk_first && epb == 0) return LSMGPU_ERR_ARG;
  if (!d_blk_first) nblocks = n ? (n + epb - 1) / epb : 1;
  if (nblocks == 0) return LSMGPU_ERR_ARG;
  uint64_t data_len = 10 * n + key_total + vs_total + 13 * nblocks;
  uint64_t total = data_len + 4 * nblocks + 4;
  if (data_len > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  if (total > out_cap) return LSMGPU_ERR_CAPACITY;
  HIPC(hipSetDevice(c->device));
  EncodeParams p{};
  p.keys = d_keys;
  p.key_end = d_key_end;
  p.vs = d_vs;
  p.vs_end = d_vs_end;
  p.n = n;
  p.epb = epb;
  p.blk_first = d_blk_first;
  p.nblocks = (uint32_t)nblocks;
  p.key_total = key_total;
  p.vs_total = vs_total;
  p.out = d_out;
  p.data_len = data_len;
  p.flags = d_flags;
  p.pad = c->flags.as<uint8_t>() + 128;  // 16 readable bytes (encode_pipe_kernel)
  HIPC(launch_encode(p, c->num_cus, c->stream));
  return LSMGPU_OK;
}

int lsmgpu_encode_blocks(lsmgpu_ctx* c, const uint8_t* keys, const uint32_t* key_end,
                         const uint8_t* vs, const uint32_t* vs_end, uint64_t n, int on_device,
                         uint32_t epb, uint32_t block_bytes, uint8_t* out, uint64_t out_cap,
                         uint64_t* out_len, uint64_t* data_len, uint32_t* restarts,
                         uint64_t restarts_cap, uint64_t* nrestarts) {
  if (!out_len) return LSMGPU_ERR_ARG;
  // out == NULL is a size query: only key_end / vs_end are read (host arrays; a NULL ctx is
  // allowed then), *out_len / *data_len / *nrestarts are filled and nothing is encoded
  const bool query = out == nullptr;
  if (n && (!key_end || !vs_end)) return LSMGPU_ERR_ARG;
  if (!query && (!c || (n && (!keys || !vs)))) return LSMGPU_ERR_ARG;
  if (query && on_device && !c) return LSMGPU_ERR_ARG;
  if (epb == 0 && block_bytes == 0) return LSMGPU_ERR_ARG;
  if (c) HIPC(hipSetDevice(c->device));
  SyncOnExit sync_exit;
  if (c) sync_exit.s[0] = c->stream;
  // host copies of the offset columns (needed for totals and the byte-target plan)
  std::vector<uint32_t> hk, hv;
  const uint32_t* hke = key_end;
  const uint32_t* hve = vs_end;
  if (on_device && n) {
    hk.resize(n);
    hv.resize(n);
    HIPC(hcopy(c, hk.data(), key_end, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(hcopy(c, hv.data(), vs_end, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    hke = hk.data();
    hve = hv.data();
  }
  const uint64_t key_total = n ? hke[n - 1] : 0, vs_total = n ? hve[n - 1] : 0;
  for (uint64_t e = 0; e < n; e++) {  // host-side validation (also flagged on device)
    uint64_t kl = hke[e] - (e ? hke[e - 1] : 0), vl = hve[e] - (e ? hve[e - 1] : 0);
    if (kl <= 8 || kl > 0xffff) return LSMGPU_ERR_KEY_LEN;
    if (vl > 0xffff) return LSMGPU_ERR_VALUE_LEN;
  }
  uint64_t nb = 0;
  std::vector<uint32_t> plan;
  const bool explicit_plan = block_bytes > 0;
  if (explicit_plan) {
    int rc = lsmgpu_plan_blocks(hke, hve, n, epb, block_bytes, nullptr, 0, &nb);
    if (rc != LSMGPU_OK) return rc;
    plan.resize(nb + 1);
    rc = lsmgpu_plan_blocks(hke, hve, n, epb, block_bytes, plan.data(), nb + 1, &nb);
    if (rc != LSMGPU_OK) return rc;
  } else {
    nb = n ? (n + epb - 1) / epb : 1;
  }
  const uint64_t dl = 10 * n + key_total + vs_total + 13 * nb;
  const uint64_t total = dl + 4 * nb + 4;
  *out_len = total;
  if (data_len) *data_len = dl;
  if (nrestarts) *nrestarts = nb;
  if (dl > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  if (query) return LSMGPU_OK;
  if (total > out_cap) return LSMGPU_ERR_CAPACITY;

  const uint8_t* dk = keys;
  const uint32_t* dke = key_end;
  const uint8_t* dv = vs;
  const uint32_t* dve = vs_end;
  uint8_t* dout = out;
  if (!on_device) {
    HIPC(c->s_a.ensure(key_total + 16));
    HIPC(c->s_b.ensure(n * 4 + 16));
    HIPC(c->s_c.ensure(vs_total + 16));
    HIPC(c->s_d.ensure(n * 4 + 16));
    HIPC(c->s_kd.ensure(total + 16));
    if (key_total) HIPC(hcopy(c, c->s_a.p, keys, key_total, hipMemcpyHostToDevice, c->stream));
    if (vs_total) HIPC(hcopy(c, c->s_c.p, vs, vs_total, hipMemcpyHostToDevice, c->stream));
    if (n) {
      HIPC(hcopy(c, c->s_b.p, key_end, n * 4, hipMemcpyHostToDevice, c->stream));
      HIPC(hcopy(c, c->s_d.p, vs_end, n * 4, hipMemcpyHostToDevice, c->stream));
    }
    dk = c->s_a.as<uint8_t>();
    dke = c->s_b.as<uint32_t>();
    dv = c->s_c.as<uint8_t>();
    dve = c->s_d.as<uint32_t>();
    dout = c->s_kd.as<uint8_t>();
  }
  const uint32_t* dplan = nullptr;
  if (explicit_plan) {
    HIPC(c->s_bf.ensure((nb + 1) * 4));
    HIPC(hcopy(c, c->s_bf.p, plan.data(), (nb + 1) * 4, hipMemcpyHostToDevice, c->stream));
    dplan = c->s_bf.as<uint32_t>();
  }
  HIPC(hipMemsetAsync(c->flags.p, 0, 16, c->stream));
  int rc = lsmgpu_encode_blocks_async(c, dk, dke, dv, dve, n, epb, dplan, nb, key_total, vs_total,
                                      dout, total, c->flags.as<uint32_t>());
  if (rc != LSMGPU_OK) return rc;
  uint32_t hflags[4] = {0, 0, 0, 0};
  HIPC(hcopy(c, hflags, c->flags.p, 16, hipMemcpyDeviceToHost, c->stream));
  if (!on_device) HIPC(hcopy(c, out, dout, total, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (hflags[0] & 1) return LSMGPU_ERR_KEY_LEN;
  if (hflags[0] & 2) return LSMGPU_ERR_VALUE_LEN;
  if (restarts) {
    if (nb > restarts_cap) return LSMGPU_ERR_CAPACITY;
    std::vector<uint8_t> idx(4 * nb);
    if (on_device) {
      HIPC(hcopy(c, idx.data(), out + dl, 4 * nb, hipMemcpyDeviceToHost, c->stream));
      HIPC(hipStreamSynchronize(c->stream));
    } else {
      std::memcpy(idx.data(), out + dl, 4 * nb);
    }
    for (uint64_t b = 0; b < nb; b++) restarts[b] = rd_be32(idx.data() + 4 * b);
  }
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ ValueStruct columns
int lsmgpu_encode_values(lsmgpu_ctx* c, const uint8_t* meta, const uint8_t* user_meta,
                         const uint64_t* expires_at, const uint8_t* values,
                         const uint32_t* value_end, uint64_t n, int on_device, uint8_t* vs,
                         uint64_t vs_cap, uint32_t* vs_end, uint64_t* vs_len) {
  if (!c || !vs_len) return LSMGPU_ERR_ARG;
  *vs_len = 0;
  if (n == 0) return LSMGPU_OK;
  if (!meta || !user_meta || !expires_at || !value_end || !vs || !vs_end) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  SyncOnExit sync_exit;
  sync_exit.s[0] = c->stream;
  uint64_t vtotal = 0;
  if (on_device) {
    uint32_t last = 0;
    HIPC(hcopy(c, &last, value_end + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    vtotal = last;
  } else {
    vtotal = value_end[n - 1];
  }
  if (!values && vtotal) return LSMGPU_ERR_ARG;
  ValuesParams p{};
  p.n = n;
  if (on_device) {
    p.meta = meta; p.user_meta = user_meta; p.expires_at = expires_at; p.values = values;
    p.value_end = value_end; p.vs = vs; p.vs_end = vs_end;
  } else {
    HIPC(c->s_a.ensure(n * 2 + 16));
    HIPC(c->s_b.ensure(n * 8 + 16));
    HIPC(c->s_c.ensure(vtotal + 16));
    HIPC(c->s_d.ensure(n * 4 + 16));
    HIPC(c->s_ve.ensure(n * 4 + 16));
    uint8_t* dm = c->s_a.as<uint8_t>();
    HIPC(hcopy(c, dm, meta, n, hipMemcpyHostToDevice, c->stream));
    HIPC(hcopy(c, dm + n, user_meta, n, hipMemcpyHostToDevice, c->stream));
    HIPC(hcopy(c, c->s_b.p, expires_at, n * 8, hipMemcpyHostToDevice, c->stream));
    if (vtotal) HIPC(hcopy(c, c->s_c.p, values, vtotal, hipMemcpyHostToDevice, c->stream));
    HIPC(hcopy(c, c->s_d.p, value_end, n * 4, hipMemcpyHostToDevice, c->stream));
    p.meta = dm; p.user_meta = dm + n; p.expires_at = c->s_b.as<uint64_t>();
    p.values = c->s_c.as<uint8_t>(); p.value_end = c->s_d.as<uint32_t>();
    p.vs_end = c->s_ve.as<uint32_t>();
  }
  // sizes -> scratch, inclusive scan -> vs_end (rocPRIM device scan)
  uint32_t* final_end = p.vs_end;
  HIPC(c->s_view.ensure(n * 4 + 16));
  p.vs_end = c->s_view.as<uint32_t>();
  HIPC(launch_values_sizes(p, c->stream));
  size_t tmp = 0;
  HIPC(rocprim::inclusive_scan(nullptr, tmp, p.vs_end, final_end, (size_t)n,
                               rocprim::plus<uint32_t>(), c->stream));
  HIPC(c->scan_tmp.ensure(tmp + 16));
  HIPC(rocprim::inclusive_scan(c->scan_tmp.p, tmp, p.vs_end, final_end, (size_t)n,
                               rocprim::plus<uint32_t>(), c->stream));
  p.vs_end = final_end;
  uint32_t total = 0;
  HIPC(hcopy(c, &total, p.vs_end + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  *vs_len = total;
  if (total > vs_cap) return LSMGPU_ERR_CAPACITY;
  if (!on_device) {
    HIPC(c->s_kd.ensure((uint64_t)total + 16));
    p.vs = c->s_kd.as<uint8_t>();
  }
  HIPC(launch_values_write(p, c->stream));
  if (!on_device) {
    HIPC(hcopy(c, vs, p.vs, total, hipMemcpyDeviceToHost, c->stream));
    HIPC(hcopy(c, vs_end, p.vs_end, n * 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIPC(hipStreamSynchronize(c->stream));
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ batched table open
int lsmgpu_open_tables_async(lsmgpu_ctx* c, const uint8_t* d_data, uint64_t data_len,
                             const uint64_t* d_sst_off, const uint64_t* d_sst_len,
                             uint32_t ntables, const lsmgpu_tables* out, uint64_t* d_result) {
  if (!c || !out || !d_result) return LSMGPU_ERR_ARG;
  if (ntables && (!d_data || !d_sst_off || !d_sst_len)) return LSMGPU_ERR_ARG;
  if (!out->nblk || !out->blk_base || !out->bloom_off || !out->bloom_len || !out->status ||
      !out->smallest || !out->biggest)
    return LSMGPU_ERR_ARG;
  if (out->blk_cap && (!out->blk_off || !out->blk_len || !out->key_off || !out->key_len ||
                       !out->order))
    return LSMGPU_ERR_ARG;
  if (out->blk_cap > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
  if (ntables == 0) return LSMGPU_OK;
  const size_t scratch = ((size_t)ntables * 8 + 255) / 256 * 256;
  const size_t sbytes = open_scan_bytes(ntables);
  if (scratch + sbytes > c->open_tmp.cap) {
    HIPC(hipStreamSynchronize(c->stream));
    HIPC(c->open_tmp.ensure(scratch + sbytes));
  }
  OpenParams p{};
  p.data = d_data;
  p.data_len = data_len;
  p.sst_off = d_sst_off;
  p.sst_len = d_sst_len;
  p.ntables = ntables;
  p.out = *out;
  p.rpos = c->open_tmp.as<uint32_t>();
  p.flags = p.rpos + ntables;
  p.result = d_result;
  HIPC(launch_open_tables(p, c->open_tmp.as<uint8_t>() + scratch, sbytes, c->stream));
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ k-way merge
int lsmgpu_merge_runs_async(lsmgpu_ctx* c, const lsmgpu_runs* in, const lsmgpu_merged* out,
                            uint64_t* d_result) {
  if (!c || !in || !out || !d_result) return LSMGPU_ERR_ARG;
  if (in->n > 0xfffffffeull) return LSMGPU_ERR_TOO_LARGE;
  if (in->n && (!in->key_data || !in->key_end || !in->val_end || !in->run_first || in->nruns == 0))
    return LSMGPU_ERR_ARG;
  if (out->val_data && !in->val_data) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
  const uint32_t n = (uint32_t)in->n;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t dst_b = al((size_t)n * 4 + 4), flg_b = 256;
  const size_t tb_b = al(((size_t)in->nruns + 1) * 4);
  const size_t spl_b = al(((size_t)n / 256 + in->nruns) * in->nruns * 4 + 4);
  const size_t rec_b = al((size_t)n * 16 + 16);
  const size_t nch = ((size_t)n + kMergeEmitTile - 1) / kMergeEmitTile;
  const size_t occ_b = al(nch * 128 + 16), cpre_b = al(nch * 4 + 4), drop_b = al((size_t)n + 1);
  const size_t need = dst_b + flg_b + tb_b + spl_b + rec_b + occ_b + cpre_b + drop_b;
  if (need > c->merge_tmp.cap) {
    HIPC(hipStreamSynchronize(c->stream));
    HIPC(c->merge_tmp.ensure(need));
  }
  // emit tile records share the decode's look-back scratch (epoch-tagged, stream-ordered):
  // [ticket u32, padded to 256 B][64 B per tile]
  const size_t lb_need = 256 + ((size_t)n / 256 + 1) * 64;  // emit tiles of >= 256 positions
  if (lb_need > c->lb.cap) {
    HIPC(hipStreamSynchronize(c->stream));
    HIPC(c->lb.ensure(lb_need));
    HIPC(hipMemset(c->lb.p, 0, c->lb.cap));
  }
  next_tag(c, 0);
  uint8_t* w = c->merge_tmp.as<uint8_t>();
  MergeParams p{};
  p.kd = in->key_data;
  p.ke = in->key_end;
  p.vd = in->val_data;
  p.ve = in->val_end;
  p.run_first = in->run_first;
  p.nruns = in->nruns;
  p.n = n;
  p.dst = reinterpret_cast<uint32_t*>(w);
  p.flags = reinterpret_cast<uint32_t*>(w + dst_b);
  p.tile_base = reinterpret_cast<uint32_t*>(w + dst_b + flg_b);
  p.spl = reinterpret_cast<uint32_t*>(w + dst_b + flg_b + tb_b);
  uint8_t* w2 = w + dst_b + flg_b + tb_b + spl_b;
  p.rec = reinterpret_cast<uint4*>(w2);
  p.occ = reinterpret_cast<uint32_t*>(w2 + rec_b);
  p.cpre = reinterpret_cast<uint32_t*>(w2 + rec_b + occ_b);
  p.drop = w2 + rec_b + occ_b + cpre_b;
  p.gcnt = c->lb.as<uint32_t>();
  p.lb = reinterpret_cast<uint64_t*>(c->lb.as<uint8_t>() + 256);
  p.tag = c->tag;
  p.okd = out->key_data;
  p.key_cap = out->key_cap;
  p.oke = out->key_end;
  p.ovd = out->val_data;
  p.val_cap = out->val_cap;
  p.ove = out->val_end;
  p.osrc = out->src;
  p.ent_cap = out->ent_cap;
  p.result = d_result;
  HIPC(launch_merge(p, c->stream));
  return LSMGPU_OK;
}

// ------------------------------------------------------------------ compaction output tables
int lsmgpu_cut_tables_async(lsmgpu_ctx* c, const uint32_t* d_key_end, const uint32_t* d_vs_end,
                            uint64_t n, uint32_t entries_per_block, int64_t cap,
                            uint32_t* d_tbl_first, uint32_t* d_tbl_blk, uint64_t* d_tbl_out,
                            uint32_t tables_cap, uint64_t* d_result) {
  return lsmgpu_cut_tables_ex_async(c, d_key_end, d_vs_end, n, entries_per_block, cap, 0,
                                    d_tbl_first, d_tbl_blk, d_tbl_out, tables_cap, d_result);
}

int lsmgpu_cut_tables_ex_async(lsmgpu_ctx* c, const uint32_t* d_key_end, const uint32_t* d_vs_end,
                               uint64_t n, uint32_t entries_per_block, int64_t cap, uint32_t flags,
                               uint32_t* d_tbl_first, uint32_t* d_tbl_blk, uint64_t* d_tbl_out,
                               uint32_t tables_cap, uint64_t* d_result) {
  if (flags & ~(uint32_t)LSMGPU_CUT_BLOOM) return LSMGPU_ERR_ARG;
  if (!c || !d_tbl_first || !d_tbl_blk || !d_tbl_out || !d_result) return LSMGPU_ERR_ARG;
  if (n && (!d_key_end || !d_vs_end)) return LSMGPU_ERR_ARG;
  if (entries_per_block == 0 || tables_cap == 0) return LSMGPU_ERR_ARG;
  if (n > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemsetAsync(d_result, 0, 8 * sizeof(uint64_t), c->stream));
  CutParams p{};
  p.key_end = d_key_end;
  p.vs_end = d_vs_end;
  p.n = n;
  p.epb = entries_per_block;
  p.cap = cap;
  p.tbl_first = d_tbl_first;
  p.tbl_blk = d_tbl_blk;
  p.tbl_out = d_tbl_out;
  p.tables_cap = tables_cap;
  p.result = d_result;
  p.bloom = (flags & LSMGPU_CUT_BLOOM) != 0;
  p.logw = std::log(0.01);
  p.ln2 = 0.69314718056;
  volatile double l2 = p.ln2 * p.ln2;  // math.Pow(0.69314718056, 2): one rounded product
  p.ln2sq = l2;
  HIPC(launch_cut_tables(p, c->stream));
  return LSMGPU_OK;
}

namespace {
int encode_tables_impl(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                  const uint8_t* d_vs, const uint32_t* d_vs_end, const uint32_t* d_src,
                  const uint32_t* d_out_key_end, const uint32_t* d_out_vs_end, uint64_t n,
                  uint64_t key_total, uint64_t vs_total, uint32_t entries_per_block,
                  const uint32_t* d_tbl_first, const uint32_t* d_tbl_blk,
                  const uint64_t* d_tbl_out, uint32_t tables_cap, uint64_t max_blocks,
                  uint8_t* d_out, uint32_t* d_flags) {
  if (!c || !d_tbl_first || !d_tbl_blk || !d_tbl_out || !d_out || !d_flags) return LSMGPU_ERR_ARG;
  if (n && (!d_keys || !d_key_end || !d_vs || !d_vs_end)) return LSMGPU_ERR_ARG;
  if (n && d_src && (!d_out_key_end || !d_out_vs_end)) return LSMGPU_ERR_ARG;
  if (entries_per_block == 0 || tables_cap == 0) return LSMGPU_ERR_ARG;
  if (max_blocks > 0xffffffffull || n > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  if (n == 0) return LSMGPU_OK;
  HIPC(hipSetDevice(c->device));
  EncodeParams p{};
  p.keys = d_keys;
  p.vs = d_vs;
  if (d_src) {  // gather: placed by the merged ends, bytes read at the source entries
    p.key_end = d_out_key_end;
    p.vs_end = d_out_vs_end;
    p.src = d_src;
    p.src_key_end = d_key_end;
    p.src_vs_end = d_vs_end;
  } else {
    p.key_end = d_key_end;
    p.vs_end = d_vs_end;
  }
  p.n = n;
  p.key_total = key_total;
  p.vs_total = vs_total;
  p.epb = entries_per_block;
  p.nblocks = (uint32_t)max_blocks;
  p.out = d_out;
  p.flags = d_flags;
  p.tbl_first = d_tbl_first;
  p.tbl_blk = d_tbl_blk;
  p.tbl_out = d_tbl_out;
  p.ntables = tables_cap;  // the kernel reads the real count from the arrays' closing entries
  p.pad = c->flags.as<uint8_t>() + 128;  // 16 readable bytes (encode_pipe_kernel)
  HIPC(launch_encode(p, c->num_cus, c->stream));
  return LSMGPU_OK;
}
}  // namespace

int lsmgpu_encode_tables_async(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                               const uint8_t* d_vs, const uint32_t* d_vs_end, uint64_t n,
                               uint64_t key_total, uint64_t vs_total,
                               uint32_t entries_per_block, const uint32_t* d_tbl_first,
                               const uint32_t* d_tbl_blk, const uint64_t* d_tbl_out,
                               uint32_t tables_cap, uint64_t max_blocks, uint8_t* d_out,
                               uint32_t* d_flags) {
  return encode_tables_impl(c, d_keys, d_key_end, d_vs, d_vs_end, nullptr, nullptr, nullptr, n,
                       key_total, vs_total, entries_per_block, d_tbl_first, d_tbl_blk, d_tbl_out,
                       tables_cap, max_blocks, d_out, d_flags);
}

int lsmgpu_encode_tables_gather_async(lsmgpu_ctx* c, const uint8_t* d_keys,
                                      const uint32_t* d_key_end, const uint8_t* d_vs,
                                      const uint32_t* d_vs_end, const uint32_t* d_src,
                                      const uint32_t* d_out_key_end, const uint32_t* d_out_vs_end,
                                      uint64_t n, uint64_t key_total, uint64_t vs_total,
                                      uint32_t entries_per_block, const uint32_t* d_tbl_first,
                                      const uint32_t* d_tbl_blk, const uint64_t* d_tbl_out,
                                      uint32_t tables_cap, uint64_t max_blocks, uint8_t* d_out,
                                      uint32_t* d_flags) {
  if (n && !d_src) return LSMGPU_ERR_ARG;
  return encode_tables_impl(c, d_keys, d_key_end, d_vs, d_vs_end, d_src, d_out_key_end, d_out_vs_end,
                       n, key_total, vs_total, entries_per_block, d_tbl_first, d_tbl_blk,
                       d_tbl_out, tables_cap, max_blocks, d_out, d_flags);
}

}  // extern "C"


// ---- bloom tail (table/builder.go:164-195, table/table.go:180-186,301; bloom.hip)
namespace {
// bbloom.New(n, 0.01): calcSizeByWrongPositives + getSize (float64 exactly as Go evaluates it)
void bloom_size(uint64_t key_count, uint64_t* bits, uint64_t* locs, uint32_t* exponent) {
  const double n = (double)key_count, ln2 = 0.69314718056;
  volatile double l2 = ln2 * ln2;  // math.Pow(0.69314718056, 2): one rounded product
  const double size = -1 * n * std::log(0.01) / l2;
  const double lc = std::ceil(ln2 * size / n);
  *locs = std::isnan(lc) ? (1ull << 63) : (uint64_t)lc;  // Go's uint64(NaN) on amd64
  uint64_t entries = (uint64_t)size, sz = 1;
  uint32_t e = 0;
  if (entries < 512) entries = 512;
  while (sz < entries) {
    sz <<= 1;
    e++;
  }
  *bits = sz;
  *exponent = e;
}
int bloom_text(uint64_t set_locs, char* text, uint32_t* head, uint32_t* tail) {
  static const char kHead[] = "{\"FilterSet\":\"";
  *head = sizeof kHead - 1;
  memcpy(text, kHead, *head);
  const int t = snprintf(text + *head, 64 - *head, "\",\"SetLocs\":%llu}",
                         (unsigned long long)set_locs);
  if (t <= 0 || *head + (uint32_t)t + 4 > 64) return LSMGPU_ERR_INTERNAL;  // room for a BE32
  *tail = (uint32_t)t;
  return LSMGPU_OK;
}
uint32_t log2_pow2(uint64_t bits) {
  uint32_t e = 0;
  while ((1ull << e) < bits) e++;
  return e;
}
bool bloom_bits_ok(uint64_t bits) { return bits >= 512 && (bits & (bits - 1)) == 0 && bits <= (1ull << 40); }
}  // namespace

int lsmgpu_bloom_params(uint64_t key_count, uint64_t* bits, uint64_t* set_locs, uint64_t* json_len) {
  if (!bits || !set_locs) return LSMGPU_ERR_ARG;
  uint32_t e = 0;
  bloom_size(key_count, bits, set_locs, &e);
  if (json_len) {
    char text[64];
    uint32_t h = 0, t = 0;
    const int rc = bloom_text(*set_locs, text, &h, &t);
    if (rc != LSMGPU_OK) return rc;
    *json_len = h + 4 * ((*bits / 8 + 2) / 3) + t;
  }
  return LSMGPU_OK;
}

int lsmgpu_bloom_build_async(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                             uint64_t n, uint64_t* d_bitset, uint64_t bits, uint64_t set_locs,
                             uint32_t* d_flags) {
  if (!c || !d_bitset || !d_flags || !bloom_bits_ok(bits)) return LSMGPU_ERR_ARG;
  if (n && (!d_keys || !d_key_end)) return LSMGPU_ERR_ARG;
  if (n > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemsetAsync(d_bitset, 0, bits / 8, c->stream));
  HIPC(hipMemsetAsync(d_flags, 0, sizeof(uint32_t), c->stream));
  BloomParams p{};
  p.keys = d_keys;
  p.key_end = d_key_end;
  p.n = n;
  p.bitset = d_bitset;
  p.mask = bits - 1;
  p.locs = set_locs;
  p.shift = 64 - log2_pow2(bits);
  p.flags = d_flags;
  HIPC(launch_bloom_build(p, c->stream));
  return LSMGPU_OK;
}

int lsmgpu_bloom_json_async(lsmgpu_ctx* c, const uint64_t* d_bitset, uint64_t bits,
                            uint64_t set_locs, uint8_t* d_out, uint64_t out_cap) {
  if (!c || !d_bitset || !d_out || !bloom_bits_ok(bits)) return LSMGPU_ERR_ARG;
  BloomJson j{};
  uint32_t h = 0, t = 0;
  const int rc = bloom_text(set_locs, reinterpret_cast<char*>(j.text), &h, &t);
  if (rc != LSMGPU_OK) return rc;
  j.bitset = d_bitset;
  j.nbytes = bits / 8;
  j.out = d_out;
  j.head_len = h;
  j.tail_len = t;
  if (out_cap < h + 4 * ((j.nbytes + 2) / 3) + t) return LSMGPU_ERR_CAPACITY;
  HIPC(hipSetDevice(c->device));
  HIPC(launch_bloom_json(j, c->stream));
  return LSMGPU_OK;
}

int lsmgpu_bloom_has_async(lsmgpu_ctx* c, const uint64_t* d_bitset, uint64_t bits,
                           uint64_t set_locs, const uint8_t* d_keys, const uint32_t* d_key_end,
                           uint64_t n, uint8_t* d_has) {
  if (!c || !d_bitset || !bloom_bits_ok(bits)) return LSMGPU_ERR_ARG;
  if (n && (!d_keys || !d_key_end || !d_has)) return LSMGPU_ERR_ARG;
  if (n > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  HIPC(hipSetDevice(c->device));
  BloomParams p{};
  p.keys = d_keys;
  p.key_end = d_key_end;
  p.n = n;
  p.bitset = const_cast<uint64_t*>(d_bitset);
  p.mask = bits - 1;
  p.locs = set_locs;
  p.shift = 64 - log2_pow2(bits);
  p.has = d_has;
  HIPC(launch_bloom_has(p, c->stream));
  return LSMGPU_OK;
}

namespace {
int bloom_tables_impl(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                 const uint32_t* d_src, const uint32_t* tbl_first, const uint64_t* tbl_out,
                 uint32_t ntables, uint8_t* d_out, uint64_t* d_scratch, uint64_t scratch_words,
                 uint32_t* d_flags);
}  // namespace

int lsmgpu_bloom_tables_async(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                              const uint32_t* tbl_first, const uint64_t* tbl_out, uint32_t ntables,
                              uint8_t* d_out, uint64_t* d_scratch, uint64_t scratch_words,
                              uint32_t* d_flags) {
  return bloom_tables_impl(c, d_keys, d_key_end, nullptr, tbl_first, tbl_out, ntables, d_out,
                      d_scratch, scratch_words, d_flags);
}

int lsmgpu_bloom_tables_gather_async(lsmgpu_ctx* c, const uint8_t* d_keys,
                                     const uint32_t* d_key_end, const uint32_t* d_src,
                                     const uint32_t* tbl_first, const uint64_t* tbl_out,
                                     uint32_t ntables, uint8_t* d_out, uint64_t* d_scratch,
                                     uint64_t scratch_words, uint32_t* d_flags) {
  if (ntables && !d_src) return LSMGPU_ERR_ARG;
  return bloom_tables_impl(c, d_keys, d_key_end, d_src, tbl_first, tbl_out, ntables, d_out, d_scratch,
                      scratch_words, d_flags);
}

namespace {
int bloom_tables_impl(lsmgpu_ctx* c, const uint8_t* d_keys, const uint32_t* d_key_end,
                 const uint32_t* d_src, const uint32_t* tbl_first, const uint64_t* tbl_out,
                 uint32_t ntables, uint8_t* d_out, uint64_t* d_scratch, uint64_t scratch_words,
                 uint32_t* d_flags) {
  if (!c || !tbl_first || !tbl_out || !d_out || !d_scratch || !d_flags) return LSMGPU_ERR_ARG;
  if (ntables && (!d_keys || !d_key_end)) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemsetAsync(d_flags, 0, sizeof(uint32_t), c->stream));
  // up to kBloomSegs tables per launch pair, their filters side by side in the scratch
  for (uint32_t t0 = 0; t0 < ntables; t0 += kBloomSegs) {
    const uint32_t nseg = std::min<uint32_t>(kBloomSegs, ntables - t0);
    BloomTables p{};
    p.keys = d_keys;
    p.key_end = d_key_end;
    p.src = d_src;
    p.scratch = d_scratch;
    p.out = d_out;
    p.flags = d_flags;
    p.nseg = nseg;
    p.end = tbl_first[t0 + nseg];
    uint64_t words = 0, groups = 0;
    for (uint32_t k = 0; k < nseg; k++) {
      const uint32_t t = t0 + k;
      const uint64_t cnt = tbl_first[t + 1] - tbl_first[t];
      if (cnt == 0 || tbl_first[t + 1] < tbl_first[t] || tbl_out[t + 1] < tbl_out[t])
        return LSMGPU_ERR_ARG;
      uint64_t bits = 0, locs = 0, jl = 0;
      int rc = lsmgpu_bloom_params(cnt, &bits, &locs, &jl);
      if (rc != LSMGPU_OK) return rc;
      if (tbl_out[t + 1] - tbl_out[t] < jl + 4 || locs > 0xffffffffull) return LSMGPU_ERR_CAPACITY;
      BloomSeg& sg = p.seg[k];
      sg.word_off = words;
      sg.mask = bits - 1;
      sg.json_out = tbl_out[t + 1] - jl - 4;
      sg.group_off = groups;
      sg.first = tbl_first[t];
      sg.shift = 64 - log2_pow2(bits);
      sg.locs = (uint32_t)locs;
      const int tl = snprintf(reinterpret_cast<char*>(sg.tail), sizeof sg.tail, "\",\"SetLocs\":%llu}",
                              (unsigned long long)locs);
      if (tl <= 0 || (uint32_t)tl + 4 > sizeof sg.tail) return LSMGPU_ERR_INTERNAL;
      for (int b = 0; b < 4; b++) sg.tail[tl + b] = (uint8_t)(jl >> (24 - 8 * b));  // bloomLen
      sg.tail_len = (uint32_t)tl + 4;
      words += bits / 64;
      groups += (bits / 8 + 2) / 3;
    }
    if (words > scratch_words) return LSMGPU_ERR_CAPACITY;
    HIPC(hipMemsetAsync(d_scratch, 0, words * 8, c->stream));
    HIPC(launch_bloom_tables(p, groups, c->stream));
  }
  return LSMGPU_OK;
}
}  // namespace


// ---- whole-compaction data path (levels.go:239-298 compactBuildTables) for host tables
namespace {
int compact_fail(lsmgpu_ctx* c, int rc) {
  c->cp_valid = false;
  return rc;
}
}  // namespace

extern "C" int lsmgpu_compact_tables(lsmgpu_ctx* c, const uint8_t* const* ssts,
                                     const uint64_t* sst_len, uint32_t ntables,
                                     const uint32_t* run_first, uint32_t nruns,
                                     int64_t max_table_size, uint32_t flags, uint64_t* out_len,
                                     uint32_t* out_tables) {
  if (!c || !out_len || !out_tables) return LSMGPU_ERR_ARG;
  *out_len = 0;
  *out_tables = 0;
  c->cp_valid = false;
  if (flags & ~(uint32_t)LSMGPU_COMPACT_BLOOM) return LSMGPU_ERR_ARG;
  if (ntables && (!ssts || !sst_len)) return LSMGPU_ERR_ARG;
  if (!run_first || nruns == 0 || run_first[0] != 0 || run_first[nruns] != ntables)
    return LSMGPU_ERR_ARG;
  for (uint32_t r = 0; r < nruns; r++)
    if (run_first[r + 1] < run_first[r]) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  SyncOnExit sync_exit;
  sync_exit.s[0] = c->stream;
  // 1. every table's tail (Table.readIndex, table.go:177-215) -> one block list over the
  //    concatenated data regions; run r starts at block rblk[r]
  std::vector<uint32_t> off, len;
  std::vector<uint64_t> base(ntables + 1, 0);
  std::vector<uint32_t> tblk(ntables + 1, 0);
  uint32_t max_len = 0;
  for (uint32_t t = 0; t < ntables; t++) {
    if (!ssts[t]) return LSMGPU_ERR_ARG;
    uint64_t nb = 0, bo = 0, bl = 0;
    int rc = lsmgpu_parse_index(ssts[t], sst_len[t], nullptr, nullptr, 0, &nb, &bo, &bl);
    if (rc != LSMGPU_OK && rc != LSMGPU_ERR_CAPACITY) return rc;
    const size_t at = off.size();
    off.resize(at + nb);
    len.resize(at + nb);
    rc = lsmgpu_parse_index(ssts[t], sst_len[t], off.data() + at, len.data() + at, nb, &nb, &bo, &bl);
    if (rc != LSMGPU_OK) return rc;
    const uint64_t dend = nb ? (uint64_t)off[at + nb - 1] + len[at + nb - 1] : 0;
    for (uint64_t i = at; i < at + nb; i++) {
      if (base[t] + off[i] > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
      off[i] += (uint32_t)base[t];
      max_len = std::max(max_len, len[i]);
    }
    base[t + 1] = base[t] + dend;
    tblk[t + 1] = (uint32_t)off.size();
  }
  const uint64_t data_len = base[ntables];
  if (data_len > 0xffffffffull) return LSMGPU_ERR_TOO_LARGE;
  // 2. inputs to HBM, one decode over every block of every input (materialize)
  HIPC(c->cp_data.ensure(data_len + 64));
  for (uint32_t t = 0; t < ntables; t++)
    if (base[t + 1] > base[t])
      HIPC(hcopy(c, c->cp_data.as<uint8_t>() + base[t], ssts[t], base[t + 1] - base[t],
                          hipMemcpyHostToDevice, c->stream));
  HIPC(c->cp_res.ensure(64));
  uint64_t* d_res = c->cp_res.as<uint64_t>();
  uint64_t r[8];
  // one materialize decode of the block list (o, l); blk_first / blk_status come back to bf / bs
  std::vector<uint32_t> bf, bs;
  auto decode_list = [&](const std::vector<uint32_t>& o, const std::vector<uint32_t>& l) -> int {
    const uint64_t nb = o.size();
    HIPC(c->cp_off.ensure(nb * 4 + 4));
    HIPC(c->cp_len.ensure(nb * 4 + 4));
    if (nb) {
      HIPC(hcopy(c, c->cp_off.p, o.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
      HIPC(hcopy(c, c->cp_len.p, l.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
    }
    uint64_t kcap = std::max<uint64_t>(data_len, 16), vcap = kcap, ecap = data_len / 10 + 1;
    for (int attempt = 0;; attempt++) {  // plen > 0 blocks can expand keys: resize once
      HIPC(c->cp_kd.ensure(kcap + 16));
      HIPC(c->cp_vd.ensure(vcap + 16));
      HIPC(c->cp_ke.ensure(ecap * 4 + 4));
      HIPC(c->cp_ve.ensure(ecap * 4 + 4));
      HIPC(c->cp_bf.ensure(nb * 4 + 4));
      HIPC(c->cp_bs.ensure(nb * 4 + 4));
      lsmgpu_decoded d{};
      d.key_data = c->cp_kd.as<uint8_t>();
      d.key_cap = kcap;
      d.key_end = c->cp_ke.as<uint32_t>();
      d.val_data = c->cp_vd.as<uint8_t>();
      d.val_cap = vcap;
      d.val_end = c->cp_ve.as<uint32_t>();
      d.ent_cap = ecap;
      d.blk_first = c->cp_bf.as<uint32_t>();
      d.blk_status = c->cp_bs.as<int32_t>();
      int rc = lsmgpu_decode_blocks_async(c, c->cp_data.as<uint8_t>(), data_len,
                                          c->cp_off.as<uint32_t>(), c->cp_len.as<uint32_t>(), nb,
                                          max_len, LSMGPU_MODE_MATERIALIZE, &d, d_res);
      if (rc != LSMGPU_OK) return rc;
      HIPC(hcopy(c, r, d_res, 64, hipMemcpyDeviceToHost, c->stream));
      HIPC(hipStreamSynchronize(c->stream));
      if (r[5] & 2) return LSMGPU_ERR_INTERNAL;
      if (!(r[5] & 1)) break;
      if (attempt) return LSMGPU_ERR_CAPACITY;
      kcap = std::max<uint64_t>(r[1], 16);
      vcap = std::max<uint64_t>(r[2], 16);
      ecap = std::max<uint64_t>(r[0], 1);
    }
    bf.assign(nb + 1, 0);
    bs.assign(nb + 1, 0);
    HIPC(hcopy(c, bf.data(), c->cp_bf.p, (nb + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    if (nb) HIPC(hcopy(c, bs.data(), c->cp_bs.p, nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return LSMGPU_OK;
  };
  int drc = decode_list(off, len);
  if (drc != LSMGPU_OK) return drc;
  // Which decoded entries Go's iterators reach (levels.go:243-253, table/iterator.go:183,
  // 201-217,301-326,412-496, y/iterator.go:128-147): tables were opened by OpenTable first.
  const int32_t kOk = LSMGPU_BLK_OK, kVo = LSMGPU_BLK_VALUE_OVERFLOW;
  std::vector<uint8_t> rewind_ok(ntables, 0), visited(ntables, 0);
  for (uint32_t t = 0; t < ntables; t++) {
    const uint32_t b0 = tblk[t], b1 = tblk[t + 1];
    for (uint32_t b = b0; b < b1; b++) {
      const uint32_t nb = bf[b + 1] - bf[b];
      const int32_t st = bs[b];
      // readIndex asserts plen == 0 on every block's first header (table.go:239): log.Fatal
      if (nb == 0 && st == LSMGPU_BLK_FIRST_PLEN) return LSMGPU_ERR_CORRUPT;
      // a terminator-first block of a multi-block table: readIndex's sort compares its empty
      // first key (table.go:267 -> y.CompareKeys' len > 8 assertion, y.go:85)
      if (nb == 0 && st == kOk && len[b] >= 10 && b1 - b0 >= 2) return LSMGPU_ERR_CORRUPT;
      // NewIterator runs block 0's first Next (iterator.go:183): a truncated first header panics
      if (b == b0 && nb == 0 && st == LSMGPU_BLK_TRUNC_HEADER) return LSMGPU_ERR_CORRUPT;
    }
    // Rewind = seekToFirst: valid only when block 0 yields an entry (iterator.go:201-217)
    rewind_ok[t] = b1 > b0 && bf[b0 + 1] > bf[b0];
  }
  // every run is a ConcatIterator (a single table behaves the same): its Rewind rewinds only the
  // first table -- if that one is invalid the MergeIterator drops the whole run (initHeap);
  // otherwise Next skips the later tables whose Rewind is invalid
  for (uint32_t k = 0; k < nruns; k++) {
    const uint32_t a = run_first[k], e = run_first[k + 1];
    if (a == e || !rewind_ok[a]) continue;
    for (uint32_t t = a; t < e; t++) visited[t] = rewind_ok[t];
  }
  bool filter = false;
  for (uint32_t t = 0; t < ntables; t++) {
    const uint32_t b0 = tblk[t], b1 = tblk[t + 1];
    if (!visited[t]) {
      filter = filter || bf[b1] > bf[b0];  // entries Go never reaches
      continue;
    }
    for (uint32_t b = b0; b < b1; b++) {
      // Iterator.next into a block that yields nothing returns Valid with a nil key: the merge
      // then compares it (y.CompareKeys asserts) or Value() panics in Decode (iterator.go:312-313)
      if (b != b0 && bf[b + 1] == bf[b]) return LSMGPU_ERR_CORRUPT;
      // a truncated header or a prefix past the base key panics when the iterator reaches it; a
      // value overflow ends the block after the entries before it (iterator.go:103-106,318-323)
      if (bs[b] != kOk && bs[b] != kVo) return LSMGPU_ERR_CORRUPT;
    }
  }
  if (filter) {  // rare (corrupt input): decode again without the tables Go never reaches
    std::vector<uint32_t> o2, l2;
    std::vector<uint32_t> tb2(ntables + 1, 0);
    for (uint32_t t = 0; t < ntables; t++) {
      if (visited[t])
        for (uint32_t b = tblk[t]; b < tblk[t + 1]; b++) {
          o2.push_back(off[b]);
          l2.push_back(len[b]);
        }
      tb2[t + 1] = (uint32_t)o2.size();
    }
    tblk.swap(tb2);
    drc = decode_list(o2, l2);
    if (drc != LSMGPU_OK) return drc;
  }
  const uint64_t n = r[0];
  if (n > 0xfffffffeull) return LSMGPU_ERR_TOO_LARGE;
  // 3. runs in entries: run r = the entries of tables [run_first[r], run_first[r+1])
  std::vector<uint32_t> rf(nruns + 1);
  for (uint32_t k = 0; k <= nruns; k++) rf[k] = bf[tblk[run_first[k]]];
  if (n == 0) {  // every input empty: the Go loop builds no table
    c->cp_tbl_out.assign(1, 0);
    c->cp_bytes = 0;
    c->cp_valid = true;
    return LSMGPU_OK;
  }
  HIPC(c->cp_rf.ensure((nruns + 1) * 4));
  HIPC(hcopy(c, c->cp_rf.p, rf.data(), (nruns + 1) * 4, hipMemcpyHostToDevice, c->stream));
  // 4. MergeIterator (y/iterator.go:74-202): lower run index wins ties, duplicates dropped
  // the merge writes the merged order (source index + end offsets), not the bytes: the
  // encoder reads each entry's bytes from the decoded tables, the one copy builder.Add makes
  HIPC(c->cp_msrc.ensure(n * 4 + 4));
  HIPC(c->cp_mke.ensure(n * 4 + 4));
  HIPC(c->cp_mve.ensure(n * 4 + 4));
  lsmgpu_runs runs{c->cp_kd.as<uint8_t>(), c->cp_ke.as<uint32_t>(), c->cp_vd.as<uint8_t>(),
                   c->cp_ve.as<uint32_t>(), c->cp_rf.as<uint32_t>(), nruns, n};
  lsmgpu_merged mo{nullptr, 0, c->cp_mke.as<uint32_t>(), nullptr, 0, c->cp_mve.as<uint32_t>(),
                   c->cp_msrc.as<uint32_t>(), n};
  int rc = lsmgpu_merge_runs_async(c, &runs, &mo, d_res);
  if (rc != LSMGPU_OK) return rc;
  uint64_t m[8];
  HIPC(hcopy(c, m, d_res, 64, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (m[3] & LSMGPU_MERGE_TIMEOUT) return LSMGPU_ERR_INTERNAL;
  if (m[3] & LSMGPU_MERGE_KEY_LEN) return LSMGPU_ERR_KEY_LEN;
  if (m[3] & LSMGPU_MERGE_UNSORTED) return LSMGPU_ERR_CORRUPT;
  if (m[3]) return LSMGPU_ERR_CAPACITY;
  const uint64_t mn = m[0], mk = m[1], mv = m[2];
  // 5. output tables where Builder.ReachedCapacity(max_table_size) starts a new builder
  const bool bloom = (flags & LSMGPU_COMPACT_BLOOM) != 0;
  uint64_t tcap = std::min<uint64_t>(mn, (10 * mn + mk + mv) / (uint64_t)std::max<int64_t>(max_table_size / 2, 1) + 16);
  uint64_t cut[8];
  for (int attempt = 0;; attempt++) {
    HIPC(c->cp_tf.ensure((tcap + 1) * 4));
    HIPC(c->cp_tb.ensure((tcap + 1) * 4));
    HIPC(c->cp_to.ensure((tcap + 1) * 8));
    rc = lsmgpu_cut_tables_ex_async(c, c->cp_mke.as<uint32_t>(), c->cp_mve.as<uint32_t>(), mn, 100,
                                    max_table_size, bloom ? LSMGPU_CUT_BLOOM : 0u,
                                    c->cp_tf.as<uint32_t>(), c->cp_tb.as<uint32_t>(),
                                    c->cp_to.as<uint64_t>(), (uint32_t)tcap, d_res);
    if (rc != LSMGPU_OK) return rc;
    HIPC(hcopy(c, cut, d_res, 64, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (!cut[3]) break;
    if (attempt || tcap >= mn) return LSMGPU_ERR_INTERNAL;
    tcap = mn;  // one entry per table is the most there can be
  }
  const uint32_t nt = (uint32_t)cut[0];
  const uint64_t bytes = cut[2];
  // 6. every table's image in one encode launch (+ every bloom tail)
  HIPC(c->cp_out.ensure(bytes + 16));
  HIPC(c->cp_flags.ensure(16));
  HIPC(hipMemsetAsync(c->cp_flags.p, 0, 16, c->stream));
  rc = lsmgpu_encode_tables_gather_async(c, c->cp_kd.as<uint8_t>(), c->cp_ke.as<uint32_t>(),
                                         c->cp_vd.as<uint8_t>(), c->cp_ve.as<uint32_t>(),
                                         c->cp_msrc.as<uint32_t>(), c->cp_mke.as<uint32_t>(),
                                         c->cp_mve.as<uint32_t>(), mn, mk, mv, 100,
                                         c->cp_tf.as<uint32_t>(), c->cp_tb.as<uint32_t>(),
                                         c->cp_to.as<uint64_t>(), (uint32_t)tcap,
                                         (mn + 99) / 100 + tcap, c->cp_out.as<uint8_t>(),
                                         c->cp_flags.as<uint32_t>());
  if (rc != LSMGPU_OK) return rc;
  std::vector<uint32_t> tf(nt + 1);
  c->cp_tbl_out.assign(nt + 1, 0);
  HIPC(hcopy(c, tf.data(), c->cp_tf.p, (nt + 1) * 4, hipMemcpyDeviceToHost, c->stream));
  HIPC(hcopy(c, c->cp_tbl_out.data(), c->cp_to.p, (nt + 1) * 8, hipMemcpyDeviceToHost,
                      c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (bloom) {
    uint64_t words = 8;
    for (uint32_t g = 0; g < nt; g += kBloomSegs) {
      uint64_t w = 0;
      for (uint32_t t = g; t < std::min(nt, g + kBloomSegs); t++) {
        uint64_t bits = 0, locs = 0;
        rc = lsmgpu_bloom_params(tf[t + 1] - tf[t], &bits, &locs, nullptr);
        if (rc != LSMGPU_OK) return rc;
        w += bits / 64;
      }
      words = std::max(words, w);
    }
    HIPC(c->cp_scratch.ensure(words * 8));
    rc = lsmgpu_bloom_tables_gather_async(c, c->cp_kd.as<uint8_t>(), c->cp_ke.as<uint32_t>(),
                                          c->cp_msrc.as<uint32_t>(), tf.data(),
                                          c->cp_tbl_out.data(), nt, c->cp_out.as<uint8_t>(),
                                          c->cp_scratch.as<uint64_t>(), words,
                                          c->cp_flags.as<uint32_t>() + 1);
    if (rc != LSMGPU_OK) return compact_fail(c, rc);
  }
  uint32_t fl[4];
  HIPC(hcopy(c, fl, c->cp_flags.p, 16, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if ((fl[0] & 1) || (fl[1] & 1)) return LSMGPU_ERR_KEY_LEN;
  if (fl[0] & 2) return LSMGPU_ERR_VALUE_LEN;
  c->cp_bytes = bytes;
  c->cp_valid = true;
  *out_len = bytes;
  *out_tables = nt;
  return LSMGPU_OK;
}

extern "C" int lsmgpu_compact_result(lsmgpu_ctx* c, uint8_t* out, uint64_t out_cap,
                                     uint64_t* tbl_off, uint64_t tbl_cap) {
  if (!c || !c->cp_valid) return LSMGPU_ERR_ARG;
  const uint64_t nt = c->cp_tbl_out.size() - 1;
  if (out_cap < c->cp_bytes || tbl_cap < nt + 1) return LSMGPU_ERR_CAPACITY;
  if ((c->cp_bytes && !out) || !tbl_off) return LSMGPU_ERR_ARG;
  HIPC(hipSetDevice(c->device));
  SyncOnExit sync_exit;
  sync_exit.s[0] = c->stream;
  if (c->cp_bytes)
    HIPC(hcopy(c, out, c->cp_out.p, c->cp_bytes, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  std::memcpy(tbl_off, c->cp_tbl_out.data(), (nt + 1) * 8);
  return LSMGPU_OK;
}
