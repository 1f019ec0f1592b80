"""mpi_vision_amd -- MI355X-native multiplane-image (MPI) render / plane-sweep hot path.

Drop-in for the hot-path helpers of Findeton/mpi-vision `utils.py`; see
`mpi_vision_amd.utils` and DESIGN.md.
"""
from . import utils  # noqa: F401
from .utils import *  # noqa: F401,F403

__all__ = [n for n in dir(utils) if n.endswith("_torch") or n in (
    "inv_depths", "over_composite", "mpi_from_net_output", "mpi_render_view_u8", "device", "read_file_lines", "parse_camera_lines",
    "make_intrinsics_matrix", "scale_intrinsics")]
