// Torch-aware native runtime pieces linked into `_C` (they need ATen / autograd / HIP):
//
//  * GradTracker  -- per-parameter gradient finality across microbatches (N1g), fed by a
//                    native walk of the autograd graph at every backward-segment boundary.
//  * IpcP2P       -- device-to-device pipeline tensor transport over hipIpc mappings
//                    (N1c): the receiver pulls the sender's buffer through xGMI (or the
//                    same HBM when both ranks share a device) on its own compute stream,
//                    ordered after the producer by an inter-process HIP event.
//  * IpcAllReduce -- one-shot all-reduce for small TP messages: every rank pushes an epoch
//                    flag into its peers' mapped flag arrays and reduces all ranks' slots
//                    in rank order (bounded waits, bitwise-identical results).
#pragma once

#include <pybind11/pybind11.h>

namespace smprt_torch {
void register_bindings(pybind11::module& m);
}
