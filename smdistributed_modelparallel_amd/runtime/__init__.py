"""Pipeline runtime: engine (greenlet coroutines + ack-tree backward), transport,
schedules, module registry, partitioner, patching, activation checkpointing."""
