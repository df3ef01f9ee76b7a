// pybind11 module `_smprt`: the host-side native runtime (no torch / HIP dependency,
// so it builds with g++ in seconds and loads on CPU-only hosts).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "mailbox.h"
#include "timeline.h"

namespace py = pybind11;
using namespace smprt;

PYBIND11_MODULE(_smprt, m) {
  m.doc() = "smdistributed_modelparallel_amd native host runtime";

  py::class_<TransportStats>(m, "TransportStats")
      .def_readonly("msgs_sent", &TransportStats::msgs_sent)
      .def_readonly("msgs_recv", &TransportStats::msgs_recv)
      .def_readonly("bytes_sent", &TransportStats::bytes_sent)
      .def_readonly("bytes_recv", &TransportStats::bytes_recv)
      .def_readonly("gated_sent", &TransportStats::gated_sent)
      .def_readonly("gate_wait_us", &TransportStats::gate_wait_us);

  py::class_<Mailbox>(m, "Mailbox")
      .def(py::init<int, int>())
      .def("listen", &Mailbox::listen)
      .def("connect", &Mailbox::connect, py::call_guard<py::gil_scoped_release>())
      .def(
          "send",
          [](Mailbox& mb, int dst, int64_t tid, int channel, py::bytes payload) {
            std::string s = payload;
            py::gil_scoped_release nogil;
            mb.send(dst, tid, static_cast<uint8_t>(channel), std::move(s));
          },
          py::arg("dst"), py::arg("tid"), py::arg("channel"), py::arg("payload"))
      .def(
          "send_gated",
          [](Mailbox& mb, int dst, int64_t tid, int channel, py::bytes payload, uintptr_t gate_fn, uintptr_t ctx) {
            std::string s = payload;
            py::gil_scoped_release nogil;
            mb.send_gated(dst, tid, static_cast<uint8_t>(channel), std::move(s), reinterpret_cast<GateFn>(gate_fn),
                          ctx);
          },
          py::arg("dst"), py::arg("tid"), py::arg("channel"), py::arg("payload"), py::arg("gate_fn"),
          py::arg("gate_ctx"))
      .def(
          "send_buffer",
          [](Mailbox& mb, int dst, int64_t tid, int channel, py::buffer buf) {
            py::buffer_info info = buf.request();
            std::string s(static_cast<const char*>(info.ptr), info.size * info.itemsize);
            py::gil_scoped_release nogil;
            mb.send(dst, tid, static_cast<uint8_t>(channel), std::move(s));
          })
      .def(
          "broadcast",
          [](Mailbox& mb, std::vector<int> dsts, int64_t tid, int channel, py::bytes payload) {
            std::string s = payload;
            py::gil_scoped_release nogil;
            mb.broadcast(dsts, tid, static_cast<uint8_t>(channel), s);
          })
      .def(
          "recv",
          [](Mailbox& mb, int src, int64_t tid, double timeout) {
            std::string s;
            {
              py::gil_scoped_release nogil;
              s = mb.recv(src, tid, timeout);
            }
            return py::bytes(s);
          },
          py::arg("src"), py::arg("tid"), py::arg("timeout") = -1.0)
      .def("poll", &Mailbox::poll)
      .def("has_server_message", &Mailbox::has_server_message)
      .def(
          "next_server_message",
          [](Mailbox& mb, double timeout) -> py::object {
            Message msg;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = mb.next_server_message(&msg, timeout);
            }
            if (!ok) return py::none();
            return py::make_tuple(msg.src, msg.tid, py::bytes(msg.payload));
          },
          py::arg("timeout") = 0.0)
      .def("flush", &Mailbox::flush, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &Mailbox::shutdown, py::arg("success") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("error", &Mailbox::error)
      .def("failed_rank", &Mailbox::failed_rank)
      .def("wait_error", &Mailbox::wait_error, py::arg("timeout") = -1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("stats", &Mailbox::stats)
      .def_property_readonly("rank", &Mailbox::rank)
      .def_property_readonly("world", &Mailbox::world);

  py::class_<Timeline>(m, "Timeline")
      .def(py::init<int>())
      .def("set_output", &Timeline::set_output)
      .def_property_readonly("enabled", &Timeline::enabled)
      .def_property_readonly("roctx_enabled", &Timeline::roctx_enabled)
      .def("start_step", &Timeline::start_step)
      .def("end_step", &Timeline::end_step)
      .def("record", &Timeline::record)
      .def("mark", &Timeline::mark)
      .def("range_push", &Timeline::range_push)
      .def("range_pop", &Timeline::range_pop)
      .def("now_us", &Timeline::now_us)
      .def("flush", &Timeline::flush);
}
