// RCCL point-to-point data plane for federated gossip (module p2pfl_amd._C, class RcclPlane).
//
// One process per GPU; ONE world communicator per job generation.  Weight
// transfers are issued as ncclGroupStart/End groups on a dedicated,
// high-priority comm stream: every "epoch" of the gossip schedule (see
// p2pfl_amd/communication/xgmi/data_plane.py) becomes one group holding all of
// this rank's sends and receives of that epoch, so a k-way fan-out runs on k
// xGMI links at once and ranks that push to each other at the same moment are
// matched inside one launch (no send/recv ordering deadlock).
//
// The communicator is created NON-BLOCKING (config.blocking = 0): no host call
// ever waits inside RCCL, completion is an event on the comm stream polled with
// the GIL released, asynchronous errors are polled with ncclCommGetAsyncError,
// and a peer that dies mid-transfer is handled by ncclCommAbort (the Python
// layer then rebuilds a communicator over the survivors).
//
// The reference moves weights as pickled byte strings through gRPC unary RPCs
// (reference p2pfl/communication/grpc/grpc_client.py:118-183); nothing here
// has a counterpart there.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <memory>
#include <atomic>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

std::string nccl_msg(ncclResult_t r) { return std::string(ncclGetErrorString(r)) + " (" + std::to_string(int(r)) + ")"; }

py::bytes unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error("ncclGetUniqueId: " + nccl_msg(r));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

using Clock = std::chrono::steady_clock;

struct GroupRec {
  hipEvent_t done = nullptr;
  std::vector<torch::Tensor> keep;  // buffers stay alive until the group is released
};

class RcclPlane {
 public:
  RcclPlane(const std::string& id, int nranks, int rank, int device, double init_timeout_s)
      : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(id.size() == NCCL_UNIQUE_ID_BYTES, "RcclPlane: unique id must be ", NCCL_UNIQUE_ID_BYTES, " bytes");
    TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "RcclPlane: bad rank/nranks");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    int lo = 0, hi = 0;
    hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    // highest priority: transfers are short and latency-critical next to training kernels
    hip_ok(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreateWithPriority");
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;
      r = ncclCommInitRankConfig(&comm_, nranks_, uid, rank_, &cfg);
      if (r == ncclInProgress) r = settle(init_timeout_s);
    }
    if (r != ncclSuccess) {
      if (comm_ != nullptr) ncclCommAbort(comm_);
      comm_ = nullptr;
      hipStreamDestroy(stream_);
      throw std::runtime_error("ncclCommInitRankConfig: " + nccl_msg(r));
    }
  }

  ~RcclPlane() {
    // never block at teardown: a still-connected communicator is aborted
    if (comm_ != nullptr) ncclCommAbort(comm_);
    for (auto& kv : groups_)
      if (kv.second.done) hipEventDestroy(kv.second.done);
    if (stream_) hipStreamDestroy(stream_);
  }

  // ops: (kind, peer, tensor) with kind 0 = send, 1 = recv.  The comm stream
  // first waits on every stream in `after` (the producers of the send
  // buffers / previous users of the receive buffers).  Returns a group id.
  //
  // Lock discipline (no host mutex is ever held while the GIL is taken back):
  // argument checks run under the GIL only; the RCCL group is enqueued with
  // the GIL released under issue_mu_ (one group at a time on the
  // communicator) and comm_mu_ (shared; abort takes it exclusively), both of
  // which are dropped before the GIL is re-acquired; the group's bookkeeping
  // entry is added afterwards under a short mu_ section.  wait/query/release
  // take mu_ with the GIL held, so holding mu_ across a GIL re-acquire would
  // be a lock-order inversion (issuer: mu_ -> GIL, completer: GIL -> mu_).
  int64_t issue(const std::vector<std::tuple<int64_t, int64_t, torch::Tensor>>& ops, const std::vector<int64_t>& after,
                double timeout_s) {
    TORCH_CHECK(!aborted_, "RcclPlane: communicator aborted/closed");
    for (const auto& op : ops) {
      const auto& t = std::get<2>(op);
      const int64_t peer = std::get<1>(op), kind = std::get<0>(op);
      TORCH_CHECK(kind == 0 || kind == 1, "RcclPlane: op kind must be 0 (send) or 1 (recv)");
      TORCH_CHECK(peer >= 0 && peer < nranks_, "RcclPlane: peer ", peer, " out of range");
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclPlane: buffers must be contiguous GPU tensors");
      TORCH_CHECK(t.get_device() == device_, "RcclPlane: buffer on device ", t.get_device(), ", plane on ", device_);
    }
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    for (int64_t s : after) {
      hipEvent_t ev;
      hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
      hip_ok(hipEventRecord(ev, reinterpret_cast<hipStream_t>(s)), "hipEventRecord(producer)");
      hip_ok(hipStreamWaitEvent(stream_, ev, 0), "hipStreamWaitEvent");
      hip_ok(hipEventDestroy(ev), "hipEventDestroy");
    }
    GroupRec rec;
    ncclResult_t r;
    bool gone = false;
    {
      py::gil_scoped_release nogil;
      std::lock_guard<std::mutex> il(issue_mu_);
      std::shared_lock<std::shared_mutex> cl(comm_mu_);
      if (comm_ == nullptr) {
        gone = true;
        r = ncclInvalidUsage;
      } else {
        r = ncclGroupStart();
      }
      for (const auto& op : ops) {
        if (r != ncclSuccess) break;
        const auto& t = std::get<2>(op);
        const size_t nbytes = size_t(t.numel()) * t.element_size();
        const int peer = int(std::get<1>(op));
        r = std::get<0>(op) == 0 ? ncclSend(t.data_ptr(), nbytes, ncclUint8, peer, comm_, stream_)
                                 : ncclRecv(t.data_ptr(), nbytes, ncclUint8, peer, comm_, stream_);
      }
      if (!gone) {
        ncclResult_t e = ncclGroupEnd();
        if (r == ncclSuccess) r = e;
        if (r == ncclInProgress) r = settle(timeout_s);
        // the completion event is recorded right behind the group, before
        // another issuer can enqueue on the comm stream
        if (r == ncclSuccess && hipEventCreateWithFlags(&rec.done, hipEventDisableTiming) == hipSuccess &&
            hipEventRecord(rec.done, stream_) != hipSuccess) {
          hipEventDestroy(rec.done);
          rec.done = nullptr;
        }
      }
    }
    if (gone) throw std::runtime_error("RcclPlane: communicator aborted");
    if (r != ncclSuccess) throw std::runtime_error("RcclPlane group: " + nccl_msg(r));
    TORCH_CHECK(rec.done != nullptr, "RcclPlane: could not record the group's completion event");
    for (const auto& op : ops) rec.keep.push_back(std::get<2>(op));
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t gid = next_gid_++;
    groups_.emplace(gid, std::move(rec));
    return gid;
  }

  // 1: complete, 0: still running.  Throws on an asynchronous RCCL error.
  int query(int64_t gid) {
    hipEvent_t ev = event_of(gid);
    hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return 1;
    if (e != hipErrorNotReady) hip_ok(e, "hipEventQuery");
    check_async();
    return 0;
  }

  // Poll (GIL released) until the group completes or `timeout_s` passes:
  // 1 done, 0 timed out.  Throws on an asynchronous RCCL error.
  int wait(int64_t gid, double timeout_s) {
    hipEvent_t ev = event_of(gid);
    const auto t_end = Clock::now() + std::chrono::duration<double>(timeout_s);
    std::string err;
    int done = 0;
    {
      py::gil_scoped_release nogil;
      int spins = 0;
      while (true) {
        hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) { done = 1; break; }
        if (e != hipErrorNotReady) { err = std::string("hipEventQuery: ") + hipGetErrorString(e); break; }
        ncclResult_t a = async_error_nolock();
        if (a != ncclSuccess && a != ncclInProgress) { err = "RCCL async error: " + nccl_msg(a); break; }
        if (Clock::now() >= t_end) break;
        // spin briefly (xGMI transfers of a few MB take ~100 us), then back off
        if (++spins > 200) std::this_thread::sleep_for(std::chrono::microseconds(spins > 2000 ? 200 : 20));
      }
    }
    if (!err.empty()) throw std::runtime_error(err);
    return done;
  }

  // Make `stream` wait for the group (consumers may enqueue before it is done).
  void stream_wait(int64_t gid, int64_t stream) {
    hip_ok(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), event_of(gid), 0), "hipStreamWaitEvent");
  }

  void release(int64_t gid) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = groups_.find(gid);
    if (it == groups_.end()) return;
    if (it->second.done) hipEventDestroy(it->second.done);
    groups_.erase(it);
  }

  int async_error() {
    ncclResult_t a = async_error_nolock();
    return int(a);
  }

  // Abort every in-flight operation (a peer died); the plane is unusable afterwards.
  void abort() {
    abort_req_ = true;
    py::gil_scoped_release nogil;
    std::unique_lock<std::shared_mutex> cl(comm_mu_);  // in-progress settles see abort_req_ and let go
    if (comm_ != nullptr) ncclCommAbort(comm_);
    comm_ = nullptr;
    aborted_ = true;
  }

  // Orderly shutdown after all groups completed (collective over live ranks in RCCL's view).
  // Orderly shutdown: let in-flight groups drain (bounded), then release the
  // communicator.  Abort rather than ncclCommDestroy so that teardown can never
  // wait on a peer (a rank that left early must not hang the survivors' exit).
  void close(double timeout_s) {
    py::gil_scoped_release nogil;
    const auto t_end = Clock::now() + std::chrono::duration<double>(timeout_s);
    while (hipStreamQuery(stream_) == hipErrorNotReady && Clock::now() < t_end)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    abort_req_ = true;
    std::unique_lock<std::shared_mutex> cl(comm_mu_);
    if (comm_ != nullptr) ncclCommAbort(comm_);
    comm_ = nullptr;
  }

  int64_t stream() const { return reinterpret_cast<int64_t>(stream_); }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }
  bool aborted() const { return aborted_; }
  size_t in_flight() {
    std::lock_guard<std::mutex> lk(mu_);
    return groups_.size();
  }

 private:
  hipEvent_t event_of(int64_t gid) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = groups_.find(gid);
    TORCH_CHECK(it != groups_.end(), "RcclPlane: unknown group ", gid);
    return it->second.done;
  }

  ncclResult_t async_error_nolock() {
    std::shared_lock<std::shared_mutex> cl(comm_mu_);
    if (comm_ == nullptr) return aborted_ ? ncclRemoteError : ncclSuccess;
    ncclResult_t a = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(comm_, &a);
    return r == ncclSuccess ? a : r;
  }

  void check_async() {
    ncclResult_t a = async_error_nolock();
    if (a != ncclSuccess && a != ncclInProgress) throw std::runtime_error("RCCL async error: " + nccl_msg(a));
  }

  // Non-blocking communicator: poll until the last call settles (GIL already released).
  ncclResult_t settle(double timeout_s) {
    const auto t_end = Clock::now() + std::chrono::duration<double>(timeout_s);
    ncclResult_t a = ncclInProgress;
    while (true) {
      ncclResult_t r = ncclCommGetAsyncError(comm_, &a);
      if (r != ncclSuccess) return r;
      if (a != ncclInProgress) return a;
      if (Clock::now() >= t_end || abort_req_) return ncclInProgress;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

  int nranks_, rank_, device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;                 // group bookkeeping (never held across a GIL transition)
  std::mutex issue_mu_;           // one group enqueue at a time (taken with the GIL released)
  std::shared_mutex comm_mu_;     // comm_ lifetime: shared for calls, exclusive for abort/close
  std::atomic<bool> abort_req_{false};
  std::unordered_map<int64_t, GroupRec> groups_;
  int64_t next_gid_ = 1;
  std::atomic<bool> aborted_{false};
};

}  // namespace

void register_rccl(py::module& m) {
  m.def("rccl_unique_id", &unique_id, "new RCCL unique id (bytes) for a communicator");
  m.def("rccl_version", &rccl_version, "RCCL library version code");
  py::class_<RcclPlane>(m, "RcclPlane")
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("unique_id"), py::arg("nranks"),
           py::arg("rank"), py::arg("device"), py::arg("init_timeout_s") = 120.0)
      .def("issue", &RcclPlane::issue, py::arg("ops"), py::arg("after") = std::vector<int64_t>{},
           py::arg("timeout_s") = 60.0)
      .def("query", &RcclPlane::query)
      .def("wait", &RcclPlane::wait, py::arg("gid"), py::arg("timeout_s"))
      .def("stream_wait", &RcclPlane::stream_wait)
      .def("release", &RcclPlane::release)
      .def("async_error", &RcclPlane::async_error)
      .def("abort", &RcclPlane::abort)
      .def("close", &RcclPlane::close, py::arg("timeout_s") = 10.0)
      .def("in_flight", &RcclPlane::in_flight)
      .def_property_readonly("stream", &RcclPlane::stream)
      .def_property_readonly("rank", &RcclPlane::rank)
      .def_property_readonly("nranks", &RcclPlane::nranks)
      .def_property_readonly("device", &RcclPlane::device)
      .def_property_readonly("aborted", &RcclPlane::aborted);
}
