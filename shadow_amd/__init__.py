"""shadow_amd -- MI355X-native routing-table build for the Shadow network
simulator: all-pairs shortest paths over the GML network graph
(NetworkGraph::compute_shortest_paths) and the batched per-round packet drop
decision (Worker::send_packet), as hand-written gfx950 HIP kernels behind the C
ABI in include/srt.h.

The package is a thin host-side mirror of the reference interface; all compute
runs in libsrt.so on the GPU.  There is no CPU fallback.
"""
from ._lib import SrtError, init, init_async, lib  # noqa: F401
from .graph import (IpAssignment, NetGraphError, NetworkGraph, PathProperties, PathTable,  # noqa: F401
                    RoutingInfo, generate_routing_info, load_network_graph)

__all__ = ["NetworkGraph", "PathProperties", "PathTable", "RoutingInfo", "IpAssignment", "NetGraphError",
           "SrtError", "generate_routing_info", "load_network_graph", "lib", "init", "init_async"]
