"""Drop-in module name of the reference (``from lf_das import LFProc, ...``,
low_pass_dascore.ipynb cell 1).  Re-exports lfdas.lf_das."""
from lfdas.lf_das import (LFProc, _check_merge, _down_sample_processing,  # noqa: F401
                          _get_filename, _get_timestr, get_edge_effect_time,
                          get_patch_time, waterfall_plot)
from lfdas.core import FrozenDict  # noqa: F401
