// Multi-device groups (include/meyda_gpu.h, "Multi-device groups").
//
// Buffers are independent in the reference (src/meyda.js:69-91 keeps no state from one
// buffer to the next), so a batch is cut into contiguous shards, one per device. Each
// device runs its own plan (src/meyda.js:17-97: the tables of `new Meyda(...)`) on its
// shard, chunk by chunk. A non-root rank extracts chunk c straight into one packed
// transfer buffer (structure of arrays) and sends it to the root with ncclSend on its
// communication stream while chunk c+1 is extracted on the compute stream (two buffers
// alternate); the root extracts its own shard straight into its outputs, receives every
// peer's chunk into a staging slot (ncclRecv) and scatters it into place with one small
// kernel on the communication stream. RCCL is loaded at run time (dlopen), so the library
// has no link-time dependency on it and a one-rank group never touches it.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mgx_internal.h"

using mgx::fail;
using mgx::hip_fail;

namespace {

// ------------------------------------------------------------------ RCCL loader
struct Rccl {
  bool ok = false;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  // what the communicator itself reports (mgx_group_comm_info)
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommCuDevice)(const ncclComm_t, int*) = nullptr;
};

// Loaded once per process: $MGX_RCCL_LIB, else librccl.so.1 from the loader path, else
// the ROCm installation's copy.
Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r.ok ? &r : nullptr;
  tried = true;
  void* h = nullptr;
  const char* env = getenv("MGX_RCCL_LIB");
  const char* names[] = {env, "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  for (const char* n : names)
    if (n && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
  if (!h) return nullptr;
  bool all = true;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    all = all && fn != nullptr;
  };
  sym(r.GetUniqueId, "ncclGetUniqueId");
  sym(r.CommInitRank, "ncclCommInitRank");
  sym(r.CommInitAll, "ncclCommInitAll");
  sym(r.CommDestroy, "ncclCommDestroy");
  sym(r.GroupStart, "ncclGroupStart");
  sym(r.GroupEnd, "ncclGroupEnd");
  sym(r.Send, "ncclSend");
  sym(r.Recv, "ncclRecv");
  sym(r.GetErrorString, "ncclGetErrorString");
  r.ok = all;
  // optional: they only feed the diagnostic mgx_group_comm_info, never the data path
  auto opt = [&](auto& fn, const char* name) { fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name)); };
  opt(r.CommCount, "ncclCommCount");
  opt(r.CommUserRank, "ncclCommUserRank");
  opt(r.CommCuDevice, "ncclCommCuDevice");
  return r.ok ? &r : nullptr;
}

int rccl_fail(ncclResult_t e, const char* what) {
  Rccl* r = rccl();
  return fail(MGX_E_DEVICE, "%s: %s", what, r ? r->GetErrorString(e) : "RCCL unavailable");
}

#define HIP_OK(call, what)                              \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(e_, (what));  \
  } while (0)
#define NCCL_OK(call, what)                             \
  do {                                                  \
    ncclResult_t e_ = (call);                           \
    if (e_ != ncclSuccess) return rccl_fail(e_, what);  \
  } while (0)

constexpr int kFields = 19;  // 13 scalars, loudness_specific, mfcc, amplitude, power, complex real, imag

// Bytes per frame of output array i (mgx_packed_layout numbering).
uint64_t field_bytes(const mgx_plan_desc& d, int i) {
  if (i < MGX_NUM_SCALARS) return d.scalar_f64 ? 8 : 4;
  switch (i) {
    case 13: return 4ull * d.num_bark_bands;
    case 14: return 4ull * d.num_mfcc_coeffs;
    case 15: case 16: return 4ull * (d.buffer_size / 2);
    default: return 4ull * d.buffer_size;
  }
}

bool field_in(uint32_t mask, int i) { return (mask >> (i < 18 ? i : 17)) & 1u; }

void*& field_ptr(mgx_outputs& o, int i) {
  static void* none = nullptr;
  if (i < MGX_NUM_SCALARS) return o.scalars[i];
  switch (i) {
    case 13: return reinterpret_cast<void*&>(o.loudness_specific);
    case 14: return reinterpret_cast<void*&>(o.mfcc);
    case 15: return reinterpret_cast<void*&>(o.amplitude_spectrum);
    case 16: return reinterpret_cast<void*&>(o.power_spectrum);
    case 17: return reinterpret_cast<void*&>(o.complex_real);
    case 18: return reinterpret_cast<void*&>(o.complex_imag);
    default: return none;
  }
}

uint64_t packed_layout(const mgx_plan_desc& d, uint32_t mask, uint64_t nf, uint64_t* off) {
  uint64_t at = 0;
  for (int i = 0; i < kFields; ++i) {
    if (!field_in(mask, i)) {
      if (off) off[i] = UINT64_MAX;
      continue;
    }
    if (off) off[i] = at;
    at += (field_bytes(d, i) * nf + 255) / 256 * 256;
  }
  return at;
}

// Outputs of frames [f0, ...) of a structure-of-arrays record.
mgx_outputs offset_outputs(const mgx_plan_desc& d, const mgx_outputs& o, uint32_t mask, uint64_t f0) {
  mgx_outputs r{};
  mgx_outputs src = o;
  for (int i = 0; i < kFields; ++i)
    if (field_in(mask, i) && field_ptr(src, i))
      field_ptr(r, i) = static_cast<unsigned char*>(field_ptr(src, i)) + f0 * field_bytes(d, i);
  return r;
}

mgx_outputs packed_outputs(const mgx_plan_desc& d, unsigned char* base, uint32_t mask, uint64_t nf) {
  uint64_t off[kFields];
  packed_layout(d, mask, nf, off);
  mgx_outputs r{};
  for (int i = 0; i < kFields; ++i)
    if (off[i] != UINT64_MAX) field_ptr(r, i) = base + off[i];
  return r;
}

void chunk_of(uint64_t count, uint32_t nch, uint32_t c, uint64_t* c0, uint64_t* cn) {
  mgx_shard_range(count, nch, c, c0, cn);
}

struct Member {
  uint32_t rank = 0;
  int device = 0;
  mgx_plan* plan = nullptr;
  ncclComm_t comm = nullptr;
  hipStream_t s_comp = nullptr, s_comm = nullptr;
  hipStream_t s_alt = nullptr;  // the odd chunks' extraction (see mgx_group_extract_device)
  hipEvent_t ev_start = nullptr, ev_comp_done = nullptr, ev_comm_done = nullptr;
  hipEvent_t ev_comp[2] = {nullptr, nullptr}, ev_sent[2] = {nullptr, nullptr};
  // a transfer slot's last send was recorded in ev_sent (by this call or an earlier one: a call
  // on another stream may start before the previous call's sends are done)
  bool xfer_sent[2] = {false, false};
  unsigned char* xfer = nullptr;  // non-root: 2 packed chunk buffers; root: 2 staging slots per peer
  uint64_t xfer_bytes = 0;
  float* h_frames = nullptr;       // mgx_group_extract_host: this device's shard
  uint64_t h_frames_cap = 0;
  unsigned char* h_out = nullptr;  // root, mgx_group_extract_host: the gathered outputs
  uint64_t h_out_bytes = 0;
};

int member_init(Member& m, const mgx_plan_desc& d) {
  mgx_plan_desc pd = d;
  pd.device = m.device;
  pd.flags &= ~MGX_FLAG_RESIDENT;  // (one-frame host calls on one plan: a group's calls never take that path)
  int rc = mgx_plan_create(&pd, &m.plan);
  if (rc) return rc;
  HIP_OK(hipSetDevice(m.device), "hipSetDevice");
  HIP_OK(hipStreamCreateWithFlags(&m.s_comp, hipStreamNonBlocking), "hipStreamCreate");
  HIP_OK(hipStreamCreateWithFlags(&m.s_comm, hipStreamNonBlocking), "hipStreamCreate");
  HIP_OK(hipStreamCreateWithFlags(&m.s_alt, hipStreamNonBlocking), "hipStreamCreate");
  for (hipEvent_t* e : {&m.ev_start, &m.ev_comp_done, &m.ev_comm_done, &m.ev_comp[0], &m.ev_comp[1], &m.ev_sent[0],
                        &m.ev_sent[1]})
    HIP_OK(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
  return MGX_OK;
}

void member_free(Member& m) {
  (void)hipSetDevice(m.device);
  if (m.s_comp) (void)hipStreamSynchronize(m.s_comp);  // in-flight kernels read the plan's tables
  if (m.s_comm) (void)hipStreamSynchronize(m.s_comm);
  if (m.s_alt) (void)hipStreamSynchronize(m.s_alt);
  if (m.plan) mgx_plan_destroy(m.plan);
  m.plan = nullptr;
  if (m.comm) {
    Rccl* r = rccl();
    if (r) r->CommDestroy(m.comm);
  }
  for (hipEvent_t e : {m.ev_start, m.ev_comp_done, m.ev_comm_done, m.ev_comp[0], m.ev_comp[1], m.ev_sent[0], m.ev_sent[1]})
    if (e) (void)hipEventDestroy(e);
  if (m.s_comp) (void)hipStreamDestroy(m.s_comp);
  if (m.s_comm) (void)hipStreamDestroy(m.s_comm);
  if (m.s_alt) (void)hipStreamDestroy(m.s_alt);
  if (m.xfer) (void)hipFree(m.xfer);
  if (m.h_frames) (void)hipFree(m.h_frames);
  if (m.h_out) (void)hipFree(m.h_out);
  m = Member{};
}

int ensure(unsigned char** p, uint64_t* cap, uint64_t bytes, const char* what) {
  if (*cap >= bytes) return MGX_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(p), bytes ? bytes : 1), what);
  *cap = bytes;
  return MGX_OK;
}

// ------------------------------------------------------ the cross-process test transport
// MGX_GROUP_TRANSPORT=ipc (mgx_group_create_rank): R processes, which may share one GPU, move
// every chunk through CUDA-style IPC instead of RCCL. The ranks rendezvous on a POSIX shared-memory
// mailbox named by the group id (mgx_comm_unique_id writes that name in place of an RCCL id in this
// mode); each peer publishes the hipIpcMemHandle of its transfer buffer there, the root opens it
// (hipIpcOpenMemHandle) and its unpack kernel (the RCCL path's) reads each posted chunk from the mapped
// buffer on the root's communication stream. Per peer and transfer slot the mailbox holds two sequence
// numbers: `posted` (the peer's extraction of the slot's chunk has completed) and `consumed` (the root's
// reads of it have completed), which stand in for the completion of an ncclSend / ncclRecv pair. The
// hand-over waits on the host, one chunk behind the extraction on both sides (a rehearsal transport: the
// shard, chunk, slot and unpack code of the multi-rank path across processes, on one GPU).
constexpr uint64_t kIpcMagic = 0x6D67782D69706331ull;  // "mgx-ipc1"
constexpr uint32_t kIpcMaxRanks = 64;
constexpr char kIpcTag[] = "mgx-ipc:";

struct IpcRankBox {
  hipIpcMemHandle_t handle;
  uint64_t gen;        // bumped each time the peer's transfer buffer is (re)allocated
  uint64_t posted[2];  // per transfer slot: chunks whose extraction has completed
  uint64_t consumed[2];
  int32_t device, pid;
  uint64_t joined;
};
struct IpcMail {
  uint64_t magic;
  uint32_t nranks, pad;
  IpcRankBox r[kIpcMaxRanks];
};

bool ipc_selected() {
  const char* t = getenv("MGX_GROUP_TRANSPORT");
  return t && strcmp(t, "ipc") == 0;
}

template <class T>
T ld_acq(const T* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
template <class T>
void st_rel(T* p, T v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

// Spins (pausing, then sleeping) until pred() holds or `seconds` pass; false on the deadline.
template <class Pred>
bool ipc_wait(Pred pred, double seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    if (pred()) return true;
    if (i < 4096) {
      __builtin_ia32_pause();
    } else {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return false;
      usleep(20);
    }
  }
}

double ipc_timeout_s() {
  const char* t = getenv("MGX_IPC_TIMEOUT_S");
  return t && atof(t) > 0 ? atof(t) : 60.0;
}

}  // namespace

// The cross-process mailbox of one group member (Transport::kIpc).
struct IpcLink {
  std::string name;
  IpcMail* mail = nullptr;
  uint64_t my_gen = 0;
  uint64_t seq[2] = {0, 0};  // peer: chunks posted per slot
  // root: per peer, the mapped transfer buffer, its generation and the chunks consumed per slot
  std::vector<void*> peer_buf;
  std::vector<uint64_t> peer_gen;
  std::vector<uint64_t> peer_seq;  // 2 per peer
  std::vector<hipEvent_t> copy_ev;  // root: per (peer, slot), the completion of its reads of the slot's chunk
  std::vector<uint8_t> copy_open;   // ... recorded and not yet marked consumed
};

// $MGX_GROUP_TRACE=PREFIX: host timestamps (CLOCK_MONOTONIC, shared by the processes of a host) of every step
// of a group call's hand-over, appended to PREFIX.<rank> when the call returns (tools/gather_trace.py).
struct GroupTrace {
  struct Ev { uint64_t ns; uint32_t chunk, peer; const char* tag; };
  std::vector<Ev> ev;
  const char* prefix = getenv("MGX_GROUP_TRACE");
  void operator()(const char* tag, uint32_t chunk = 0, uint32_t peer = 0) {
    if (!prefix) return;
    ev.push_back({(uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch()).count(), chunk, peer, tag});
  }
  void flush(uint32_t rank) {
    if (!prefix || ev.empty()) return;
    char path[512];
    snprintf(path, sizeof path, "%s.%u", prefix, rank);
    if (FILE* f = fopen(path, "a")) {
      for (const Ev& e : ev) fprintf(f, "%llu %u %s %u %u\n", (unsigned long long)e.ns, rank, e.tag, e.chunk, e.peer);
      fclose(f);
    }
    ev.clear();
  }
};

// How a peer's chunk reaches the root's staging slot.
enum class Transport {
  kRccl,      // ncclSend on the peer's communication stream, ncclRecv on the root's
  kCopy,      // mgx_group_create_loopback: a device copy on the root's communication stream
  kRcclSelf,  // mgx_group_create_loopback_rccl: ncclSend + ncclRecv to self on a one-rank
              // communicator, on the root's communication stream
  kIpc,       // mgx_group_create_rank with MGX_GROUP_TRANSPORT=ipc: one process per rank (the
              // ranks may share a GPU), chunks through IPC-mapped transfer buffers and a
              // shared-memory mailbox (IpcLink)
};

struct mgx_group {
  mgx_plan_desc d;
  uint32_t nranks = 0;
  bool single_process = true;
  Transport transport = Transport::kRccl;
  std::vector<Member> m;  // local ranks, in rank order
  IpcLink ipc;            // Transport::kIpc
  bool loopback() const { return transport == Transport::kCopy || transport == Transport::kRcclSelf; }  // all ranks in this process
};

namespace {

// Creates (rank 0) or joins the mailbox named by the id, and registers this rank in it.
int ipc_join(mgx_group* g, const char* id, uint32_t rank) {
  if (strncmp(id, kIpcTag, sizeof kIpcTag - 1) != 0)
    return fail(MGX_E_INVALID_ARGUMENT, "MGX_GROUP_TRANSPORT=ipc: the group id was not made by mgx_comm_unique_id in this mode");
  if (g->nranks > kIpcMaxRanks) return fail(MGX_E_UNSUPPORTED, "the IPC transport holds at most %u ranks", kIpcMaxRanks);
  IpcLink& L = g->ipc;
  // (L.name -- the name ipc_leave unlinks -- is set only once this rank has opened the mailbox: a name
  // that already existed, or never appeared, belongs to someone else and is left alone)
  const std::string name = std::string("/") + (id + sizeof kIpcTag - 1);
  const size_t bytes = sizeof(IpcMail);
  int fd = -1;
  const double tmo = ipc_timeout_s();
  if (rank == 0) {
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return fail(MGX_E_DEVICE, "shm_open(%s): %s", name.c_str(), strerror(errno));
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      return fail(MGX_E_DEVICE, "ftruncate(mailbox): %s", strerror(errno));
    }
  } else if (!ipc_wait([&] { return (fd = shm_open(name.c_str(), O_RDWR, 0600)) >= 0; }, tmo)) {
    return fail(MGX_E_DEVICE, "rank %u: the group mailbox %s never appeared", rank, name.c_str());
  }
  L.name = name;
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return fail(MGX_E_DEVICE, "mmap(mailbox): %s", strerror(errno));
  L.mail = static_cast<IpcMail*>(p);
  if (rank == 0) {
    L.mail->nranks = g->nranks;
    st_rel(&L.mail->magic, kIpcMagic);
  } else {
    // (a peer may map the file before rank 0 has initialised it: wait for the magic word)
    if (!ipc_wait([&] { return ld_acq(&L.mail->magic) == kIpcMagic; }, tmo))
      return fail(MGX_E_DEVICE, "rank %u: the group mailbox was never initialised", rank);
    if (L.mail->nranks != g->nranks) return fail(MGX_E_INVALID_ARGUMENT, "the mailbox is for %u ranks, not %u", L.mail->nranks, g->nranks);
  }
  IpcRankBox& me = L.mail->r[rank];
  me.device = g->m[0].device;
  me.pid = (int32_t)getpid();
  st_rel(&me.joined, (uint64_t)1);
  // every rank present before anyone transfers (the barrier of a communicator's creation)
  if (!ipc_wait([&] {
        for (uint32_t r = 0; r < g->nranks; ++r)
          if (!ld_acq(&L.mail->r[r].joined)) return false;
        return true;
      }, tmo))
    return fail(MGX_E_DEVICE, "rank %u: not every rank joined the group within %.0f s", rank, tmo);
  if (rank == 0) {
    L.peer_buf.assign(g->nranks, nullptr);
    L.peer_gen.assign(g->nranks, 0);
    L.peer_seq.assign(2 * (size_t)g->nranks, 0);
  }
  return MGX_OK;
}

void ipc_leave(mgx_group* g) {
  IpcLink& L = g->ipc;
  for (hipEvent_t e : L.copy_ev)
    if (e) (void)hipEventDestroy(e);
  L.copy_ev.clear();
  L.copy_open.clear();
  for (void* b : L.peer_buf)
    if (b) (void)hipIpcCloseMemHandle(b);
  L.peer_buf.clear();
  if (L.mail) munmap(L.mail, sizeof(IpcMail));
  L.mail = nullptr;
  if (!L.name.empty()) shm_unlink(L.name.c_str());  // every rank: whichever leaves first removes the name
  L.name.clear();
}

// A peer: publish its transfer buffer's handle after an allocation (before any chunk of the call
// is posted, so the root never maps a freed buffer: the root consumed every chunk of the last one).
int ipc_publish(mgx_group* g, Member& m) {
  IpcRankBox& me = g->ipc.mail->r[m.rank];
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, m.xfer), "hipIpcGetMemHandle(transfer buffer)");
  me.handle = h;
  st_rel(&me.gen, ++g->ipc.my_gen);
  return MGX_OK;
}

// A peer, before it extracts into transfer slot sl again: the root has copied the slot's last chunk.
int ipc_wait_consumed(mgx_group* g, uint32_t rank, int sl) {
  IpcLink& L = g->ipc;
  IpcRankBox& me = L.mail->r[rank];
  if (!ipc_wait([&] { return ld_acq(&me.consumed[sl]) >= L.seq[sl]; }, ipc_timeout_s()))
    return fail(MGX_E_DEVICE, "rank %u: the root did not take chunk %llu of slot %d", rank, (unsigned long long)L.seq[sl], sl);
  return MGX_OK;
}

// A peer: chunk of slot sl extracted (its event complete): post it.
// ($MGX_IPC_FAIL_RANK, a test hook: that rank never posts, so the root's wait passes its deadline)
int ipc_post(mgx_group* g, Member& m, int sl) {
  HIP_OK(hipEventSynchronize(m.ev_comp[sl]), "hipEventSynchronize(chunk)");
  ++g->ipc.seq[sl];
  const char* f = getenv("MGX_IPC_FAIL_RANK");
  if (!(f && atoi(f) == (int)m.rank)) st_rel(&g->ipc.mail->r[m.rank].posted[sl], g->ipc.seq[sl]);
  return MGX_OK;
}

// The root: peer p's chunk of slot sl, once posted (ipc_take_start: a host wait for the post, the peer's transfer
// buffer mapped when it is new). The unpack kernel then reads the chunk straight from the peer's mapped buffer
// (*src; $MGX_IPC_COPY=1: copied into the root's staging slot `dst` first, round 5's form) -- on one device the
// mapping is the same HBM, and a hipMemcpyAsync out of an IPC mapping takes the runtime's peer-copy path, ~0.5 ms
// per 52 MB step on the rehearsal box (profiles/r06_gather_breakdown.txt). ipc_take_mark records when the
// root's reads of the slot are done; ipc_take_finish, later, waits for that and marks the slot consumed so the
// peer may reuse it. Between the two the root enqueues its next chunk.
int ipc_take_start(mgx_group* g, uint32_t p, int sl, unsigned char* dst, uint64_t slot, uint64_t bytes, hipStream_t s,
                   unsigned char** src) {
  IpcLink& L = g->ipc;
  IpcRankBox& box = L.mail->r[p];
  uint64_t& want = L.peer_seq[2 * (size_t)p + sl];
  ++want;
  if (!ipc_wait([&] { return ld_acq(&box.posted[sl]) >= want; }, ipc_timeout_s()))
    return fail(MGX_E_DEVICE, "root: rank %u never posted chunk %llu of slot %d", p, (unsigned long long)want, sl);
  *src = dst;
  if (bytes) {
    const uint64_t gen = ld_acq(&box.gen);
    if (gen != L.peer_gen[p]) {  // the peer (re)allocated its transfer buffer: map the new one
      if (L.peer_buf[p]) (void)hipIpcCloseMemHandle(L.peer_buf[p]);
      L.peer_buf[p] = nullptr;
      HIP_OK(hipIpcOpenMemHandle(&L.peer_buf[p], box.handle, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      L.peer_gen[p] = gen;
    }
    unsigned char* peer = static_cast<unsigned char*>(L.peer_buf[p]) + sl * slot;
    const char* cp = getenv("MGX_IPC_COPY");
    if (cp && atoi(cp) != 0) HIP_OK(hipMemcpyAsync(dst, peer, bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync(ipc chunk)");
    else *src = peer;
  }
  return MGX_OK;
}

int ipc_take_mark(mgx_group* g, uint32_t p, int sl, hipStream_t s) {
  IpcLink& L = g->ipc;
  const size_t k = 2 * (size_t)p + sl;
  if (L.copy_ev.size() < 2 * (size_t)g->nranks) {
    L.copy_ev.resize(2 * (size_t)g->nranks, nullptr);
    L.copy_open.resize(2 * (size_t)g->nranks, 0);
  }
  if (!L.copy_ev[k]) HIP_OK(hipEventCreateWithFlags(&L.copy_ev[k], hipEventDisableTiming), "hipEventCreate(ipc take)");
  HIP_OK(hipEventRecord(L.copy_ev[k], s), "hipEventRecord(ipc take)");
  L.copy_open[k] = 1;
  return MGX_OK;
}

int ipc_take_finish(mgx_group* g, uint32_t p, int sl) {
  IpcLink& L = g->ipc;
  const size_t k = 2 * (size_t)p + sl;
  if (k >= L.copy_open.size() || !L.copy_open[k]) return MGX_OK;
  HIP_OK(hipEventSynchronize(L.copy_ev[k]), "hipEventSynchronize(ipc chunk)");
  L.copy_open[k] = 0;
  st_rel(&L.mail->r[p].consumed[sl], L.peer_seq[k]);
  return MGX_OK;
}

}  // namespace

extern "C" {

int mgx_shard_range(uint64_t total, uint32_t nranks, uint32_t rank, uint64_t* start, uint64_t* count) {
  if (!start || !count) return fail(MGX_E_INVALID_ARGUMENT, "NULL argument");
  if (nranks == 0 || rank >= nranks) return fail(MGX_E_INVALID_ARGUMENT, "rank %u of %u", rank, nranks);
  const uint64_t base = total / nranks, extra = total % nranks;
  *start = rank * base + std::min<uint64_t>(rank, extra);
  *count = base + (rank < extra ? 1 : 0);
  return MGX_OK;
}

uint64_t mgx_packed_layout(const mgx_plan_desc* desc, uint32_t mask, uint64_t num_frames, uint64_t offsets[19]) {
  if (!desc) return 0;
  return packed_layout(*desc, mask, num_frames, offsets);
}

int mgx_comm_unique_id(void* id, uint64_t id_bytes) {
  if (!id || id_bytes < sizeof(ncclUniqueId)) return fail(MGX_E_INVALID_ARGUMENT, "id buffer must hold %d bytes", MGX_COMM_ID_BYTES);
  if (ipc_selected()) {  // the test transport: the id names the group's shared-memory mailbox
    uint64_t r = 0;
    FILE* f = fopen("/dev/urandom", "rb");
    if (!f || fread(&r, sizeof r, 1, f) != 1) r = (uint64_t)getpid() * 0x9E3779B97F4A7C15ull ^ (uint64_t)time(nullptr);
    if (f) fclose(f);
    memset(id, 0, id_bytes);
    snprintf(static_cast<char*>(id), id_bytes, "%smgx_ipc_%d_%016llx", kIpcTag, (int)getpid(), (unsigned long long)r);
    return MGX_OK;
  }
  Rccl* r = rccl();
  if (!r) return fail(MGX_E_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
  ncclUniqueId u;
  NCCL_OK(r->GetUniqueId(&u), "ncclGetUniqueId");
  memcpy(id, &u, sizeof u);
  return MGX_OK;
}

int mgx_group_create(const mgx_plan_desc* desc, const int32_t* devices, uint32_t ndev, mgx_group** out) {
  if (!out) return fail(MGX_E_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!desc || !devices || ndev == 0) return fail(MGX_E_INVALID_ARGUMENT, "a descriptor and at least one device are required");
  for (uint32_t i = 0; i < ndev; ++i)
    for (uint32_t j = 0; j < i; ++j)
      if (devices[i] == devices[j]) return fail(MGX_E_INVALID_ARGUMENT, "device %d listed twice", devices[i]);
  auto* g = new mgx_group();
  g->d = *desc;
  g->nranks = ndev;
  g->single_process = true;
  g->m.resize(ndev);
  int rc = MGX_OK;
  for (uint32_t i = 0; i < ndev && !rc; ++i) {
    g->m[i].rank = i;
    g->m[i].device = devices[i];
    rc = member_init(g->m[i], *desc);
  }
  if (!rc && ndev > 1) {
    Rccl* r = rccl();
    if (!r) {
      rc = fail(MGX_E_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
    } else {
      std::vector<ncclComm_t> comms(ndev);
      std::vector<int> devs(devices, devices + ndev);
      ncclResult_t e = r->CommInitAll(comms.data(), (int)ndev, devs.data());
      if (e != ncclSuccess) rc = rccl_fail(e, "ncclCommInitAll");
      else for (uint32_t i = 0; i < ndev; ++i) g->m[i].comm = comms[i];
    }
  }
  if (rc) {
    mgx_group_destroy(g);
    return rc;
  }
  *out = g;
  return MGX_OK;
}

static int create_loopback(const mgx_plan_desc* desc, uint32_t nranks, Transport tr, mgx_group** out) {
  if (!out) return fail(MGX_E_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!desc || nranks == 0) return fail(MGX_E_INVALID_ARGUMENT, "a descriptor and at least one rank are required");
  auto* g = new mgx_group();
  g->d = *desc;
  g->nranks = nranks;
  g->single_process = true;
  g->transport = tr;
  g->m.resize(nranks);
  int rc = MGX_OK;
  for (uint32_t i = 0; i < nranks && !rc; ++i) {
    g->m[i].rank = i;
    g->m[i].device = desc->device;
    rc = member_init(g->m[i], *desc);
  }
  if (!rc && tr == Transport::kRcclSelf) {
    // one communicator of one rank on the device, held by the root: every peer's chunk is a
    // send to self matched by a receive from self
    Rccl* r = rccl();
    if (!r) {
      rc = fail(MGX_E_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
    } else {
      const int dev = desc->device;
      (void)hipSetDevice(dev);
      ncclResult_t e = r->CommInitAll(&g->m[0].comm, 1, &dev);
      if (e != ncclSuccess) rc = rccl_fail(e, "ncclCommInitAll (one rank)");
    }
  }
  if (rc) {
    mgx_group_destroy(g);
    return rc;
  }
  *out = g;
  return MGX_OK;
}

int mgx_group_create_loopback(const mgx_plan_desc* desc, uint32_t nranks, mgx_group** out) {
  return create_loopback(desc, nranks, Transport::kCopy, out);
}

int mgx_group_create_loopback_rccl(const mgx_plan_desc* desc, uint32_t nranks, mgx_group** out) {
  return create_loopback(desc, nranks, Transport::kRcclSelf, out);
}

int mgx_group_create_rank(const mgx_plan_desc* desc, const void* unique_id, uint32_t nranks, uint32_t rank,
                          mgx_group** out) {
  if (!out) return fail(MGX_E_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!desc || nranks == 0 || rank >= nranks) return fail(MGX_E_INVALID_ARGUMENT, "rank %u of %u", rank, nranks);
  if (nranks > 1 && !unique_id) return fail(MGX_E_INVALID_ARGUMENT, "unique_id is NULL");
  auto* g = new mgx_group();
  g->d = *desc;
  g->nranks = nranks;
  g->single_process = nranks == 1;
  g->m.resize(1);
  g->m[0].rank = rank;
  g->m[0].device = desc->device;
  int rc = member_init(g->m[0], *desc);
  if (!rc && nranks > 1 && ipc_selected()) {
    g->transport = Transport::kIpc;
    rc = ipc_join(g, static_cast<const char*>(unique_id), rank);
  } else if (!rc && nranks > 1) {
    Rccl* r = rccl();
    if (!r) {
      rc = fail(MGX_E_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
    } else {
      ncclUniqueId u;
      memcpy(&u, unique_id, sizeof u);
      (void)hipSetDevice(desc->device);
      ncclResult_t e = r->CommInitRank(&g->m[0].comm, (int)nranks, u, (int)rank);
      if (e != ncclSuccess) rc = rccl_fail(e, "ncclCommInitRank");
    }
  }
  if (rc) {
    mgx_group_destroy(g);
    return rc;
  }
  *out = g;
  return MGX_OK;
}

int mgx_group_destroy(mgx_group* g) {
  if (!g) return MGX_OK;
  for (Member& m : g->m) member_free(m);
  if (g->transport == Transport::kIpc) ipc_leave(g);
  delete g;
  return MGX_OK;
}

int mgx_group_info(const mgx_group* g, uint32_t* nranks, uint32_t* first_local, uint32_t* num_local) {
  if (!g) return fail(MGX_E_INVALID_ARGUMENT, "group is NULL");
  if (nranks) *nranks = g->nranks;
  if (first_local) *first_local = g->m.empty() ? 0 : g->m[0].rank;
  if (num_local) *num_local = (uint32_t)g->m.size();
  return MGX_OK;
}

int mgx_group_comm_info(const mgx_group* g, int32_t* comm_ranks, int32_t* comm_rank, int32_t* comm_device) {
  if (!g) return fail(MGX_E_INVALID_ARGUMENT, "group is NULL");
  int32_t n = -1, me = -1, dev = -1;
  const ncclComm_t c = g->m.empty() ? nullptr : g->m[0].comm;
  if (g->transport == Transport::kIpc) {  // the mailbox's own view: every rank that joined it
    n = (int32_t)g->ipc.mail->nranks;
    me = (int32_t)g->m[0].rank;
    dev = g->ipc.mail->r[me].device;
  } else if (c) {
    Rccl* r = rccl();
    int v;
    if (!r) return fail(MGX_E_UNSUPPORTED, "RCCL could not be loaded");
    if (!r->CommCount || !r->CommUserRank || !r->CommCuDevice)
      return fail(MGX_E_UNSUPPORTED, "this RCCL lacks ncclCommCount / ncclCommUserRank / ncclCommCuDevice");
    if (r->CommCount(c, &v) != ncclSuccess) return fail(MGX_E_DEVICE, "ncclCommCount failed");
    n = v;
    if (r->CommUserRank(c, &v) != ncclSuccess) return fail(MGX_E_DEVICE, "ncclCommUserRank failed");
    me = v;
    if (r->CommCuDevice(c, &v) != ncclSuccess) return fail(MGX_E_DEVICE, "ncclCommCuDevice failed");
    dev = v;
  }
  if (comm_ranks) *comm_ranks = n;
  if (comm_rank) *comm_rank = me;
  if (comm_device) *comm_device = dev;
  return MGX_OK;
}

static int group_extract(mgx_group* g, const float* const* frames, const uint64_t* counts, const mgx_outputs* root_out,
                         uint32_t mask, uint32_t nch, void* const* streams, std::vector<hipStream_t>& cs);

int mgx_group_extract_device(mgx_group* g, const float* const* frames, const uint64_t* counts,
                             const mgx_outputs* root_out, uint32_t mask, uint32_t nch, void* const* streams) {
  if (!g || !frames || !counts) return fail(MGX_E_INVALID_ARGUMENT, "NULL argument");
  std::vector<hipStream_t> cs;
  const int rc = group_extract(g, frames, counts, root_out, mask, nch, streams, cs);
  if (rc && !cs.empty()) {
    // An error after work was enqueued: chunks may still be in flight on the second compute
    // stream and the communication stream (writing the root's outputs or reading transfer
    // slots). Join them into the callers' streams, so what a caller enqueues next stays
    // ordered after them, without a host wait (a peer that never posts its half of a message
    // would make a synchronisation hang).
    for (size_t i = 0; i < g->m.size() && i < cs.size(); ++i) {
      Member& m = g->m[i];
      (void)hipSetDevice(m.device);
      if (hipEventRecord(m.ev_comp_done, m.s_alt) == hipSuccess) (void)hipStreamWaitEvent(cs[i], m.ev_comp_done, 0);
      if (hipEventRecord(m.ev_comm_done, m.s_comm) == hipSuccess) (void)hipStreamWaitEvent(cs[i], m.ev_comm_done, 0);
    }
  }
  return rc;
}

static int group_extract(mgx_group* g, const float* const* frames, const uint64_t* counts, const mgx_outputs* root_out,
                         uint32_t mask, uint32_t nch, void* const* streams, std::vector<hipStream_t>& cs) {
  if (mask & ~MGX_OUT_ALL_MASK) return fail(MGX_E_INVALID_ARGUMENT, "unknown output bits in mask 0x%x", mask);
  const mgx_plan_desc& d = g->d;
  const uint32_t R = g->nranks;
  const uint64_t N = d.buffer_size;
  std::vector<uint64_t> start(R);
  uint64_t total = 0, most = 0;
  for (uint32_t r = 0; r < R; ++r) {
    start[r] = total;
    total += counts[r];
    most = std::max(most, counts[r]);
  }
  const bool root_local = g->m[0].rank == 0;
  if (root_local) {
    if (!root_out) return fail(MGX_E_INVALID_ARGUMENT, "root outputs are NULL on the root");
    mgx_outputs chk = *root_out;
    for (int i = 0; i < kFields; ++i)
      if (field_in(mask, i) && !field_ptr(chk, i)) return fail(MGX_E_INVALID_ARGUMENT, "output %d is in the mask but NULL", i);
  }
  for (size_t i = 0; i < g->m.size(); ++i)
    if (counts[g->m[i].rank] && !frames[i]) return fail(MGX_E_INVALID_ARGUMENT, "frames of local rank %zu are NULL", i);
  // pipeline depth: about 32 Ki frames per chunk, at most 8 chunks. Each peer's
  // records cross one xGMI link to the root (200 B per frame: ~52 MB per 262,144-frame shard,
  // of the order of the shard's extraction time), so what is not overlapped is about one
  // chunk's transfer after the last extraction: 8 chunks halve that tail against 4, and the
  // chunks' kernel boundaries cost nothing on two alternating streams.
  // (a one-rank group has nothing to overlap: one chunk)
  if (nch == 0) nch = R == 1 ? 1 : (uint32_t)std::min<uint64_t>(8, std::max<uint64_t>(1, (most + 32767) / 32768));
  uint64_t cmax = 0;
  for (uint32_t r = 0; r < R; ++r) {
    uint64_t c0, cn;
    chunk_of(counts[r], nch, 0, &c0, &cn);  // chunk 0 is the largest
    cmax = std::max(cmax, cn);
  }
  const uint64_t slot = packed_layout(d, mask, cmax, nullptr);
  const bool ipc = g->transport == Transport::kIpc && R > 1;
  // buffers: non-root 2 packed chunks; root 2 staging slots per peer
  for (Member& m : g->m) {
    HIP_OK(hipSetDevice(m.device), "hipSetDevice");
    const uint64_t need = R == 1 ? 0 : (m.rank == 0 ? 2 * slot * (R - 1) : 2 * slot);
    // (IPC: the root has taken both slots' last chunks before a peer may replace the buffer it maps)
    if (ipc && m.rank != 0 && m.xfer_bytes < need)
      for (int sl = 0; sl < 2; ++sl)
        if (int rc = ipc_wait_consumed(g, m.rank, sl)) return rc;
    unsigned char* const before = m.xfer;
    int rc = ensure(&m.xfer, &m.xfer_bytes, need, "hipMalloc(transfer buffers)");
    if (rc) return rc;
    if (ipc && m.rank != 0 && m.xfer != before && (rc = ipc_publish(g, m))) return rc;
  }
  // Extraction runs on the caller's stream (or the member's own): no cross-stream wait on
  // the compute path. Transfers and the root's scatters run on the communication stream,
  // ordered after what the caller enqueued before (the scatters write the root's outputs).
  // A NULL entry of a given array is that device's default stream, as for mgx_extract_device
  // (it is the stream a caller's earlier work is on; the members' own streams are not ordered
  // with it, since they are created non-blocking).
  // Consecutive chunks alternate between that stream and the member's second compute stream:
  // the chunks are independent, so chunk c+1's workgroups take the slots chunk c's free while
  // it drains instead of starting after its last workgroup. 8 chunks of 262,144 x 1024 on one
  // stream took 9 % longer than one launch; alternating, 1 % less. Chunk c and
  // c+2 share a transfer slot and a stream, so the slot's reuse stays ordered on that stream.
  for (size_t i = 0; i < g->m.size(); ++i) cs.push_back(streams ? static_cast<hipStream_t>(streams[i]) : g->m[i].s_comp);
  for (size_t i = 0; i < g->m.size(); ++i) {
    Member& m = g->m[i];
    if (R == 1 && nch == 1) continue;
    HIP_OK(hipSetDevice(m.device), "hipSetDevice");
    HIP_OK(hipEventRecord(m.ev_start, cs[i]), "hipEventRecord");
    if (nch > 1) HIP_OK(hipStreamWaitEvent(m.s_alt, m.ev_start, 0), "hipStreamWaitEvent");
    if (R > 1) HIP_OK(hipStreamWaitEvent(m.s_comm, m.ev_start, 0), "hipStreamWaitEvent");
  }
  const bool uses_rccl = R > 1 && g->transport != Transport::kCopy && g->transport != Transport::kIpc;
  Rccl* rc_ = uses_rccl ? rccl() : nullptr;
  if (uses_rccl && !rc_) return fail(MGX_E_UNSUPPORTED, "RCCL could not be loaded");
  // one RCCL group of point-to-point calls; on an error after ncclGroupStart the group is
  // still ended (an open group would absorb the caller's next RCCL calls)
  auto p2p_group = [&](auto&& body) -> int {
    NCCL_OK(rc_->GroupStart(), "ncclGroupStart");
    const char* what = nullptr;
    const ncclResult_t e = body(what);
    const ncclResult_t e_end = rc_->GroupEnd();
    if (e != ncclSuccess) return rccl_fail(e, what);
    if (e_end != ncclSuccess) return rccl_fail(e_end, "ncclGroupEnd");
    return MGX_OK;
  };
  GroupTrace trace;
  trace("call", nch, (uint32_t)N);  // (chunks, bufferSize)
  // ($MGX_IPC_SYNC=1, for tools/gather_trace.py: round 5's hand-over, each chunk posted and taken as soon as it
  // is enqueued, the host waiting for it before the next chunk is enqueued)
  const bool ipc_sync = ipc && getenv("MGX_IPC_SYNC") && atoi(getenv("MGX_IPC_SYNC")) != 0;
  // scatter each peer's chunk c (staging slot c & 1) into the root's outputs, on its communication
  // stream (ordered after the receive / copy into that slot)
  auto unpack = [&](Member& m, uint32_t c, unsigned char* const* srcs = nullptr) -> int {
    for (uint32_t p = 1; p < R; ++p) {
      uint64_t c0, cn;
      chunk_of(counts[p], nch, c, &c0, &cn);
      if (!cn) continue;
      uint64_t off[kFields];
      packed_layout(d, mask, cn, off);
      mgx::UnpackArgs ua{};
      ua.src = srcs ? srcs[p] : m.xfer + ((uint64_t)(p - 1) * 2 + (c & 1)) * slot;
      mgx_outputs dst = offset_outputs(d, *root_out, mask, start[p] + c0);
      for (int i = 0; i < kFields; ++i) {
        if (off[i] == UINT64_MAX) continue;
        ua.src_off[ua.nseg] = off[i];
        ua.dst[ua.nseg] = field_ptr(dst, i);
        ua.dwords[ua.nseg] = field_bytes(d, i) * cn / 4;
        ++ua.nseg;
      }
      HIP_OK(mgx::launch_unpack(ua, m.s_comm), "unpack kernel launch");
    }
    return MGX_OK;
  };
  // (IPC, the root) every peer's chunk c: taken into its staging slot once posted, then scattered
  auto ipc_take_all = [&](uint32_t c) -> int {
    Member& root = g->m[0];
    HIP_OK(hipSetDevice(root.device), "hipSetDevice");
    trace("take_wait", c);
    std::vector<unsigned char*> srcs(R, nullptr);
    for (uint32_t p = 1; p < R; ++p) {
      uint64_t c0, cn;
      chunk_of(counts[p], nch, c, &c0, &cn);
      unsigned char* dst = root.xfer + ((uint64_t)(p - 1) * 2 + (c & 1)) * slot;
      if (int rc = ipc_take_start(g, p, (int)(c & 1), dst, slot, cn ? packed_layout(d, mask, cn, nullptr) : 0, root.s_comm,
                                  &srcs[p]))
        return rc;
      trace("taken", c, p);
    }
    if (int rc = unpack(root, c, srcs.data())) return rc;
    for (uint32_t p = 1; p < R; ++p)
      if (int rc = ipc_take_mark(g, p, (int)(c & 1), root.s_comm)) return rc;
    trace("unpacked", c);
    return MGX_OK;
  };
  // ... and chunk c's copies marked consumed once complete
  auto ipc_finish_all = [&](uint32_t c) -> int {
    trace("fin_wait", c);
    for (uint32_t p = 1; p < R; ++p)
      if (int rc = ipc_take_finish(g, p, (int)(c & 1))) return rc;
    trace("consumed", c);
    return MGX_OK;
  };
  struct TraceFlush {
    GroupTrace& t;
    uint32_t rank;
    ~TraceFlush() { t.flush(rank); }
  } trace_flush{trace, g->m[0].rank};
  for (uint32_t c = 0; c < nch; ++c) {
    const int sl = (int)(c & 1);
    // extraction of chunk c on every local rank
    for (size_t i = 0; i < g->m.size(); ++i) {
      Member& m = g->m[i];
      uint64_t c0, cn;
      chunk_of(counts[m.rank], nch, c, &c0, &cn);
      HIP_OK(hipSetDevice(m.device), "hipSetDevice");
      const float* src = frames[i] + c0 * N;
      const hipStream_t st = sl ? m.s_alt : cs[i];
      if (m.rank == 0) {
        if (cn) {
          const mgx_outputs o = offset_outputs(d, *root_out, mask, start[0] + c0);
          int rc = mgx_extract_device(m.plan, src, cn, &o, st);
          if (rc) return rc;
        }
        trace("enq", c);
      } else {
        if (ipc) {  // the root has copied the slot's previous chunk out (the mailbox's `consumed`)
          trace("slot_wait", c);
          if (int rc = ipc_wait_consumed(g, m.rank, sl)) return rc;
          trace("slot_free", c);
        } else if (c >= 2 || m.xfer_sent[sl]) {
          HIP_OK(hipStreamWaitEvent(st, m.ev_sent[sl], 0), "hipStreamWaitEvent");
        }
        if (cn) {
          const mgx_outputs o = packed_outputs(d, m.xfer + sl * slot, mask, cn);
          int rc = mgx_extract_device(m.plan, src, cn, &o, st);
          if (rc) return rc;
        }
        HIP_OK(hipEventRecord(m.ev_comp[sl], st), "hipEventRecord");
        HIP_OK(hipStreamWaitEvent(m.s_comm, m.ev_comp[sl], 0), "hipStreamWaitEvent");
        trace("enq", c);
        // posted once extracted (every chunk, an empty one too: the sequence stays aligned), one chunk
        // late: chunk c is enqueued before the host waits for chunk c - 1, so the device never idles on it
        if (ipc && (ipc_sync || c >= 1)) {
          const uint32_t pc = ipc_sync ? c : c - 1;
          trace("post_wait", pc);
          if (int rc = ipc_post(g, m, (int)(pc & 1))) return rc;
          trace("posted", pc);
        }
      }
    }
    if (R == 1) continue;
    if (ipc) {
      // the root, one chunk behind its own extraction: marks chunk c - 2's copies consumed (their slots go
      // back to the peers), takes chunk c - 1 from every peer and scatters it
      Member& root = g->m[0];
      if (root.rank == 0 && ipc_sync) {
        if (int rc = ipc_take_all(c)) return rc;
        if (int rc = ipc_finish_all(c)) return rc;
      } else if (root.rank == 0) {
        if (c >= 2) {
          if (int rc = ipc_finish_all(c - 2)) return rc;
        }
        if (c >= 1) {
          if (int rc = ipc_take_all(c - 1)) return rc;
        }
      }
      continue;
    } else if (g->loopback()) {
      // the test transports: each peer's chunk into the root's staging slot on the root's
      // communication stream, after the peer's extraction of it -- a device copy, or an RCCL
      // send to self matched by a receive from self on the root's one-rank communicator
      Member& root = g->m[0];
      HIP_OK(hipSetDevice(root.device), "hipSetDevice");
      for (uint32_t p = 1; p < R; ++p) {
        Member& m = g->m[p];
        uint64_t c0, cn;
        chunk_of(counts[p], nch, c, &c0, &cn);
        HIP_OK(hipStreamWaitEvent(root.s_comm, m.ev_comp[sl], 0), "hipStreamWaitEvent");
        unsigned char* dst = root.xfer + ((uint64_t)(p - 1) * 2 + sl) * slot;
        const uint64_t bytes = packed_layout(d, mask, cn, nullptr);
        if (cn && g->transport == Transport::kCopy) {
          HIP_OK(hipMemcpyAsync(dst, m.xfer + sl * slot, bytes, hipMemcpyDeviceToDevice, root.s_comm),
                 "hipMemcpyAsync(loopback chunk)");
        } else if (cn) {
          const int rc = p2p_group([&](const char*& what) {
            what = "ncclSend (self)";
            ncclResult_t e = rc_->Send(m.xfer + sl * slot, bytes, ncclUint8, 0, root.comm, root.s_comm);
            if (e != ncclSuccess) return e;
            what = "ncclRecv (self)";
            return rc_->Recv(dst, bytes, ncclUint8, 0, root.comm, root.s_comm);
          });
          if (rc) return rc;
        }
        HIP_OK(hipEventRecord(m.ev_sent[sl], root.s_comm), "hipEventRecord");
        m.xfer_sent[sl] = true;
      }
    } else {
      // transfers of chunk c (one group: in single-process mode it spans every device)
      const int rc = p2p_group([&](const char*& what) {
        for (Member& m : g->m) {
          if (m.rank == 0) {
            for (uint32_t p = 1; p < R; ++p) {
              uint64_t c0, cn;
              chunk_of(counts[p], nch, c, &c0, &cn);
              if (!cn) continue;
              unsigned char* st = m.xfer + ((uint64_t)(p - 1) * 2 + sl) * slot;
              what = "ncclRecv";
              const ncclResult_t e = rc_->Recv(st, packed_layout(d, mask, cn, nullptr), ncclUint8, (int)p, m.comm, m.s_comm);
              if (e != ncclSuccess) return e;
            }
          } else {
            uint64_t c0, cn;
            chunk_of(counts[m.rank], nch, c, &c0, &cn);
            what = "ncclSend";
            const ncclResult_t e =
                cn ? rc_->Send(m.xfer + sl * slot, packed_layout(d, mask, cn, nullptr), ncclUint8, 0, m.comm, m.s_comm)
                   : ncclSuccess;
            if (e != ncclSuccess) return e;
          }
        }
        return ncclSuccess;
      });
      if (rc) return rc;
    }
    for (Member& m : g->m) {
      HIP_OK(hipSetDevice(m.device), "hipSetDevice");
      if (m.rank != 0) {
        if (!g->loopback()) {
          HIP_OK(hipEventRecord(m.ev_sent[sl], m.s_comm), "hipEventRecord");
          m.xfer_sent[sl] = true;
        }
        continue;
      }
      if (int rc = unpack(m, c)) return rc;
    }
  }
  if (ipc && !ipc_sync) {
    // the last chunk: the peers post it, the root finishes the hand-over (every slot consumed when the
    // call returns, so a peer's next call never waits on this one)
    for (Member& m : g->m) {
      if (m.rank == 0) continue;
      trace("post_wait", nch - 1);
      if (int rc = ipc_post(g, m, (int)((nch - 1) & 1))) return rc;
      trace("posted", nch - 1);
    }
    if (g->m[0].rank == 0) {
      int rc = nch >= 2 ? ipc_finish_all(nch - 2) : MGX_OK;
      if (!rc) rc = ipc_take_all(nch - 1);
      if (!rc) rc = ipc_finish_all(nch - 1);
      if (rc) return rc;
    }
  }
  // the callers' streams (or the members' own) wait for the odd chunks and the gather
  for (size_t i = 0; i < g->m.size(); ++i) {
    Member& m = g->m[i];
    if (R == 1 && nch == 1) break;
    HIP_OK(hipSetDevice(m.device), "hipSetDevice");
    if (nch > 1) {
      HIP_OK(hipEventRecord(m.ev_comp_done, m.s_alt), "hipEventRecord");
      HIP_OK(hipStreamWaitEvent(cs[i], m.ev_comp_done, 0), "hipStreamWaitEvent");
    }
    if (R > 1 && g->loopback() && m.rank != 0) {  // its chunks leave on the root's stream
      for (uint32_t sl = 0; sl < std::min<uint32_t>(nch, 2); ++sl)
        HIP_OK(hipStreamWaitEvent(cs[i], m.ev_sent[sl], 0), "hipStreamWaitEvent");
    } else if (R > 1) {
      HIP_OK(hipEventRecord(m.ev_comm_done, m.s_comm), "hipEventRecord");
      HIP_OK(hipStreamWaitEvent(cs[i], m.ev_comm_done, 0), "hipStreamWaitEvent");
    }
  }
  return MGX_OK;
}

int mgx_group_extract_host(mgx_group* g, const float* frames, uint64_t nframes, const mgx_outputs* o) {
  if (!g || !o) return fail(MGX_E_INVALID_ARGUMENT, "NULL group or outputs");
  if (!g->single_process || g->m.size() != g->nranks)
    return fail(MGX_E_UNSUPPORTED, "host batches need a single-process group (mgx_group_create)");
  if (nframes == 0) return MGX_OK;
  if (!frames) return fail(MGX_E_INVALID_ARGUMENT, "frames is NULL");
  if ((o->complex_real == nullptr) != (o->complex_imag == nullptr))
    return fail(MGX_E_INVALID_ARGUMENT, "complex_real and complex_imag must be given together");
  const mgx_plan_desc& d = g->d;
  const uint32_t R = g->nranks;
  const uint64_t N = d.buffer_size;
  mgx_outputs oh = *o;
  uint32_t mask = 0;
  for (int i = 0; i < 18; ++i)
    if (field_ptr(oh, i)) mask |= 1u << i;
  std::vector<uint64_t> start(R), cnt(R);
  for (uint32_t r = 0; r < R; ++r) mgx_shard_range(nframes, R, r, &start[r], &cnt[r]);
  // shards to the devices, one host thread per device (parallel PCIe copies)
  std::vector<int> rcs(R, MGX_OK);
  std::vector<std::string> errs(R);
  std::vector<std::thread> th;
  for (uint32_t r = 0; r < R; ++r) {
    th.emplace_back([&, r]() {
      Member& m = g->m[r];
      int rc = MGX_OK;
      hipError_t e = hipSetDevice(m.device);
      uint64_t cap = m.h_frames_cap * 4;
      unsigned char* p = reinterpret_cast<unsigned char*>(m.h_frames);
      if (e == hipSuccess) rc = ensure(&p, &cap, cnt[r] * N * 4, "hipMalloc(shard frames)");
      m.h_frames = reinterpret_cast<float*>(p);
      m.h_frames_cap = cap / 4;
      if (e == hipSuccess && !rc && cnt[r])
        e = hipMemcpy(m.h_frames, frames + start[r] * N, cnt[r] * N * 4, hipMemcpyHostToDevice);
      if (e != hipSuccess) rc = hip_fail(e, "hipMemcpy(shard frames)");
      if (rc) errs[r] = mgx_last_error();
      rcs[r] = rc;
    });
  }
  for (auto& t : th) t.join();
  for (uint32_t r = 0; r < R; ++r)
    if (rcs[r]) return fail(rcs[r], "%s", errs[r].c_str());
  // the gathered record on the root device
  Member& root = g->m[0];
  HIP_OK(hipSetDevice(root.device), "hipSetDevice");
  uint64_t off[kFields];
  const uint64_t bytes = packed_layout(d, mask, nframes, off);
  int rc = ensure(&root.h_out, &root.h_out_bytes, bytes, "hipMalloc(gathered outputs)");
  if (rc) return rc;
  mgx_outputs dev = packed_outputs(d, root.h_out, mask, nframes);
  std::vector<const float*> fr(R);
  for (uint32_t r = 0; r < R; ++r) fr[r] = g->m[r].h_frames;
  rc = mgx_group_extract_device(g, fr.data(), cnt.data(), &dev, mask, 0, nullptr);
  if (rc) return rc;
  for (Member& m : g->m) {
    HIP_OK(hipSetDevice(m.device), "hipSetDevice");
    HIP_OK(hipStreamSynchronize(m.s_comp), "hipStreamSynchronize");
  }
  HIP_OK(hipSetDevice(root.device), "hipSetDevice");
  for (int i = 0; i < kFields; ++i) {
    if (off[i] == UINT64_MAX) continue;
    HIP_OK(hipMemcpy(field_ptr(oh, i), root.h_out + off[i], field_bytes(d, i) * nframes, hipMemcpyDeviceToHost),
           "hipMemcpy(outputs)");
  }
  return MGX_OK;
}

}  // extern "C"
