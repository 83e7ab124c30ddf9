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
      std::lock_guard<std::mutex> nl(nccl_mu_);
      r = ncclCommInitRankConfig(&comm_, nranks_, uid, rank_, &cfg);
      if (r == ncclInProgress) r = settle(init_timeout_s);
      if (r != ncclSuccess) {
        if (comm_ != nullptr) ncclCommAbort(comm_);
        comm_ = nullptr;
      }
    }
    if (r != ncclSuccess) {
      hipStreamDestroy(stream_);
      stream_ = nullptr;
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
  // Threading (the data plane issues from one thread and completes from
  // another):
  //  * no RCCL or HIP call is made while holding the GIL -- a call that blocks
  //    inside the runtime must never stall every Python thread;
  //  * no host mutex is held across a GIL re-acquire (mu_ guards only the
  //    group table, in short sections taken with the GIL held);
  //  * every RCCL call on the communicator is serialised by nccl_mu_.  With a
  //    non-blocking communicator ncclGroupEnd hands the group to a job thread,
  //    and ncclCommGetAsyncError may *join* that job: two threads polling it
  //    concurrently (issuer settling its group, completer checking for
  //    errors) would both join one thread.  The completer therefore only
  //    try-locks nccl_mu_ to poll for asynchronous errors and skips the poll
  //    while a group is being issued.
  int64_t issue(const std::vector<std::tuple<int64_t, int64_t, torch::Tensor>>& ops, const std::vector<int64_t>& after,
                double timeout_s) {
    TORCH_CHECK(!aborted_, "RcclPlane: communicator aborted/closed");
    struct RawOp {
      int kind, peer;
      void* ptr;
      size_t nbytes;
    };
    std::vector<RawOp> raw;
    GroupRec rec;
    for (const auto& op : ops) {
      const auto& t = std::get<2>(op);
      const int64_t peer = std::get<1>(op), kind = std::get<0>(op);
      TORCH_CHECK(kind == 0 || kind == 1, "RcclPlane: op kind must be 0 (send) or 1 (recv)");
      TORCH_CHECK(peer >= 0 && peer < nranks_, "RcclPlane: peer ", peer, " out of range");
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclPlane: buffers must be contiguous GPU tensors");
      TORCH_CHECK(t.get_device() == device_, "RcclPlane: buffer on device ", t.get_device(), ", plane on ", device_);
      raw.push_back({int(kind), int(peer), t.data_ptr(), size_t(t.numel()) * t.element_size()});
      rec.keep.push_back(t);  // buffers stay alive until the group is released
    }
    ncclResult_t r = ncclSuccess;
    bool gone = false;
    std::string herr;
    {
      py::gil_scoped_release nogil;
      std::lock_guard<std::mutex> nl(nccl_mu_);
      if (comm_ == nullptr) {
        gone = true;
      } else {
        auto hcheck = [&](hipError_t e, const char* what) {
          if (e != hipSuccess && herr.empty()) herr = std::string(what) + ": " + hipGetErrorString(e);
          return e == hipSuccess;
        };
        hcheck(hipSetDevice(device_), "hipSetDevice");
        for (int64_t s : after) {
          if (!herr.empty()) break;
          hipEvent_t ev;
          if (!hcheck(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate")) break;
          if (hcheck(hipEventRecord(ev, reinterpret_cast<hipStream_t>(s)), "hipEventRecord(producer)"))
            hcheck(hipStreamWaitEvent(stream_, ev, 0), "hipStreamWaitEvent");
          hipEventDestroy(ev);
        }
        if (herr.empty()) {
          r = ncclGroupStart();
          for (const auto& op : raw) {
            if (r != ncclSuccess) break;
            r = op.kind == 0 ? ncclSend(op.ptr, op.nbytes, ncclUint8, op.peer, comm_, stream_)
                             : ncclRecv(op.ptr, op.nbytes, ncclUint8, op.peer, comm_, stream_);
          }
          ncclResult_t e = ncclGroupEnd();
          if (r == ncclSuccess) r = e;
          if (r == ncclInProgress) r = settle(timeout_s);
          // the completion event is recorded right behind the group, before
          // another group can be enqueued on the comm stream
          if (r == ncclSuccess && hcheck(hipEventCreateWithFlags(&rec.done, hipEventDisableTiming), "hipEventCreate") &&
              !hcheck(hipEventRecord(rec.done, stream_), "hipEventRecord(done)")) {
            hipEventDestroy(rec.done);
            rec.done = nullptr;
          }
        }
      }
    }
    if (gone) throw std::runtime_error("RcclPlane: communicator aborted");
    if (!herr.empty()) throw std::runtime_error("RcclPlane: " + herr);
    if (r != ncclSuccess) throw std::runtime_error("RcclPlane group: " + nccl_msg(r));
    TORCH_CHECK(rec.done != nullptr, "RcclPlane: could not record the group's completion event");
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t gid = next_gid_++;
    groups_.emplace(gid, std::move(rec));
    return gid;
  }

  // 1: complete, 0: still running.  Throws on an asynchronous RCCL error.
  int query(int64_t gid) {
    hipEvent_t ev = event_of(gid);
    hipError_t e;
    ncclResult_t a = ncclSuccess;
    {
      py::gil_scoped_release nogil;
      e = hipEventQuery(ev);
      if (e == hipErrorNotReady) a = poll_async_error();
    }
    if (e == hipSuccess) return 1;
    if (e != hipErrorNotReady) hip_ok(e, "hipEventQuery");
    if (a != ncclSuccess && a != ncclInProgress) throw std::runtime_error("RCCL async error: " + nccl_msg(a));
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
        if ((spins & 15) == 0) {
          ncclResult_t a = poll_async_error();
          if (a != ncclSuccess && a != ncclInProgress) { err = "RCCL async error: " + nccl_msg(a); break; }
        }
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
    hipEvent_t ev = event_of(gid);
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev, 0);
    }
    hip_ok(e, "hipStreamWaitEvent");
  }

  void release(int64_t gid) {
    GroupRec rec;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = groups_.find(gid);
      if (it == groups_.end()) return;
      rec = std::move(it->second);
      groups_.erase(it);
    }
    if (rec.done) hipEventDestroy(rec.done);
    // rec.keep (the transfer buffers) is dropped here, with the GIL held
  }

  int async_error() {
    py::gil_scoped_release nogil;
    return int(poll_async_error());
  }

  // Abort every in-flight operation (a peer died); the plane is unusable afterwards.
  void abort() {
    abort_req_ = true;
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> nl(nccl_mu_);  // an in-progress settle sees abort_req_ and lets go
    if (comm_ != nullptr) ncclCommAbort(comm_);
    comm_ = nullptr;
    aborted_ = true;
  }

  // Orderly shutdown: let in-flight groups drain (bounded), then release the
  // communicator.  Abort rather than ncclCommDestroy so that teardown can never
  // wait on a peer (a rank that left early must not hang the survivors' exit).
  void close(double timeout_s) {
    py::gil_scoped_release nogil;
    const auto t_end = Clock::now() + std::chrono::duration<double>(timeout_s);
    while (stream_ && hipStreamQuery(stream_) == hipErrorNotReady && Clock::now() < t_end)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    abort_req_ = true;
    std::lock_guard<std::mutex> nl(nccl_mu_);
    if (comm_ != nullptr) ncclCommAbort(comm_);
    comm_ = nullptr;
    aborted_ = true;
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

  // Asynchronous error of the communicator without ever blocking: while a
  // group is being issued (nccl_mu_ held) the poll is skipped (InProgress).
  ncclResult_t poll_async_error() {
    std::unique_lock<std::mutex> nl(nccl_mu_, std::try_to_lock);
    if (!nl.owns_lock()) return ncclInProgress;
    if (comm_ == nullptr) return aborted_ ? ncclRemoteError : ncclSuccess;
    ncclResult_t a = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(comm_, &a);
    return r == ncclSuccess ? a : r;
  }

  // Non-blocking communicator: poll until the last call settles (GIL released,
  // nccl_mu_ held by the caller).
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
  std::mutex mu_;        // group table (short sections, GIL held, never across a GIL transition)
  std::mutex nccl_mu_;   // every RCCL call on comm_ (taken with the GIL released)
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
