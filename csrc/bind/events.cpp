// Device-scope stream events for the engines' cross-stream ordering.
//
// torch.cuda.Event / Stream.wait_stream record HIP events with the default system-scope
// release: every record behind a kernel writes back the XCD L2s before the marker completes.
// On the engine's critical path (update -> next rollout chain, rollout -> GAE) those markers
// only order GPU work against GPU work, so an agent-scope release is enough
// (hipEventDisableSystemFence). Host waits still work (the completion signal is host-visible);
// what a device-scope event does NOT promise is that data the GPU wrote to host memory before it
// is visible to the host -- record a torch event for pinned D2H copies the host reads.
#include "common.h"

namespace {

class DeviceEvent {
 public:
  explicit DeviceEvent(bool device_scope) {
    unsigned flags = hipEventDisableTiming;
    if (device_scope) flags |= hipEventDisableSystemFence;
    TORCH_CHECK(hipEventCreateWithFlags(&ev_, flags) == hipSuccess, "hipEventCreateWithFlags failed");
    device_scope_ = device_scope;
  }
  ~DeviceEvent() {
    if (ev_) (void)hipEventDestroy(ev_);
  }
  DeviceEvent(const DeviceEvent&) = delete;
  DeviceEvent& operator=(const DeviceEvent&) = delete;

  // stream: a torch.cuda.Stream's cuda_stream handle, or 0 / None for the current stream
  void record(c10::optional<int64_t> stream) {
    TORCH_CHECK(hipEventRecord(ev_, pick(stream)) == hipSuccess, "hipEventRecord failed");
  }
  void wait(c10::optional<int64_t> stream) {
    TORCH_CHECK(hipStreamWaitEvent(pick(stream), ev_, 0) == hipSuccess, "hipStreamWaitEvent failed");
  }
  void synchronize() {
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = hipEventSynchronize(ev_);
    }
    TORCH_CHECK(e == hipSuccess, "hipEventSynchronize failed: ", hipGetErrorString(e));
  }
  bool query() {
    const hipError_t e = hipEventQuery(ev_);
    if (e == hipErrorNotReady) return false;
    TORCH_CHECK(e == hipSuccess, "hipEventQuery failed: ", hipGetErrorString(e));
    return true;
  }
  bool device_scope() const { return device_scope_; }

 private:
  // None: the current stream; an explicit handle as given (0 = the null stream, which is torch's
  // default stream -- not "the current stream", which inside a `with th.cuda.stream(side)` block is
  // the side stream)
  static hipStream_t pick(c10::optional<int64_t> stream) {
    if (stream.has_value()) return reinterpret_cast<hipStream_t>(*stream);
    return ia_stream();
  }
  hipEvent_t ev_ = nullptr;
  bool device_scope_ = true;
};

}  // namespace

void register_events(py::module& m) {
  py::class_<DeviceEvent>(m, "DeviceEvent")
      .def(py::init<bool>(), py::arg("device_scope") = true)
      .def("record", &DeviceEvent::record, py::arg("stream") = py::none())
      .def("wait", &DeviceEvent::wait, py::arg("stream") = py::none())
      .def("synchronize", &DeviceEvent::synchronize)
      .def("query", &DeviceEvent::query)
      .def_property_readonly("device_scope", &DeviceEvent::device_scope);
}
