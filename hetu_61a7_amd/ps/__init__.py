"""Single-node parameter server (shared-memory van) and HET embedding cache."""
from .worker import PSAgent, worker_init, worker_finish, get_agent
from .server import server_init, server_finish, scheduler_init, scheduler_finish
from .cstable import CacheSparseTable
