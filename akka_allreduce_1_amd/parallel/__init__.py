"""Distributed data plane: xGMI communicators, RCCL baseline, bucketed DP gradient reducer."""
from .comm import CommError, LocalCluster, XgmiCommunicator, free_port, init_distributed  # noqa: F401
from .ddp import BucketedGradReducer, TorchDistComm, bucket_sizes, compute_stream_excluding  # noqa: F401,E402
from .hierarchical import HierarchicalCommunicator  # noqa: F401,E402
from .p2p import P2PCommunicator, block_bounds, reduce_rows  # noqa: F401,E402
from .zero import ShardedDataParallel  # noqa: F401,E402
from .sdma import LocalSdmaCluster, SdmaCommunicator  # noqa: F401,E402
