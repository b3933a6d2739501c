"""Single-node parameter server (shared-memory van) and HET embedding cache."""

# PS key namespaces, disjoint by construction (node ids stay below 2^20):
#   [0, 2^20)              one key per graph node (embedding / PS-held tables)
#   [2^20, 2^21)           OptimizerOp flat dense buffers (PS / Hybrid modes)
#   [2^21, 2^22)           HetPipe per-stage dense buffers
#   [2^22, 2^23)           explicit parameterServerCommunicate_op dense keys
PS_KEY_OPT_FLAT = 1 << 20
PS_KEY_HETPIPE_STAGE = 1 << 21
PS_KEY_DENSE_COMM = 1 << 22
from .worker import PSAgent, worker_init, worker_finish, get_agent
from .server import server_init, server_finish, scheduler_init, scheduler_finish
from .cstable import CacheSparseTable
