"""gflownet_spai_amd — MI355X-native hot path of SPAI-via-GFlowNet (tonylizza/gflownet-spai).

Drop-in replacements for the reference's ``PreconditionerEnv`` (preconditioner.py),
``GFlowNet`` (gflownet/gflownet.py), ``Log`` (gflownet/log.py), ``ForwardPolicy`` /
``BackwardPolicy`` (policy.py) and ``trajectory_balance_loss`` (gflownet/utils.py),
backed by hand-written gfx950 kernels in ``libspai_hip.so`` (C ABI: include/spai_hip.h).
"""
from .env import Env
from .gflownet import GFlowNet
from .log import Log
from .policy import BackwardPolicy, ForwardPolicy
from .preconditioner import Data, PreconditionerEnv
from .gmres import solve_with_gmres, spai_power_pattern
from .utils import (axial_pattern_3d, load_mtx_file, lu_candidate_matrix, market_matrix_to_sparse_tensor, poisson_2d, poisson_3d,
                    thermal_like,
                    trajectory_balance_loss)

__all__ = ["Env", "GFlowNet", "Log", "ForwardPolicy", "BackwardPolicy", "PreconditionerEnv", "Data",
           "trajectory_balance_loss", "market_matrix_to_sparse_tensor", "load_mtx_file", "lu_candidate_matrix",
           "solve_with_gmres", "spai_power_pattern", "poisson_2d", "poisson_3d", "axial_pattern_3d", "thermal_like"]
