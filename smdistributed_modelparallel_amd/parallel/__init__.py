"""Data-parallel / sharding / memory machinery: flat buffers, bucketed reducer,
sharded data parallelism, activation offloading, delayed init, TP RNG."""
