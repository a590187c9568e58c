"""Data-parallel runtime: communicators, per-parameter strategies (2A/2B), bucketed DDP (3)."""
from .comm import (init_distributed_setup, test_distributed_setup, destroy,  # noqa: F401
                   TorchCommunicator, RcclCommunicator, make_communicator, SUM, AVG, MAX)
from .strategies import (sync_gradients_gather_scatter, sync_gradients_allreduce,  # noqa: F401
                         sync_gradients_gather_broadcast, STRATEGIES)
from .ddp import DistributedDataParallel, plan_buckets, check_replicas  # noqa: F401
