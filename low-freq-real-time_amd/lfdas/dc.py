"""``import lfdas.dc as dc`` — the DASCore names the reference's hot path uses
(``dc.Patch``, ``dc.spool``, ``dc.to_datetime64``, ``dc.units.s``, example
data)."""
from . import units  # noqa: F401
from .core import (Patch, Spool, get_example_patch, get_example_spool,  # noqa: F401
                   spool, to_datetime64, to_timedelta64)
