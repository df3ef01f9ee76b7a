"""Framework-agnostic backend: config, topology, object collectives, splitter, logging."""
