"""*(DASCore, external)* ``dascore.units``: the time quantities the rolling
notebooks build their windows from (rolling_mean_dascore_edge.ipynb cell 1,
``from dascore.units import s``; cell 7, ``window = d_t*s``).  DASCore uses
pint; only the time units the hot path takes are restated here."""

_SECONDS = {"s": 1.0, "ms": 1e-3, "us": 1e-6, "ns": 1e-9, "minute": 60.0, "hour": 3600.0}


class Quantity:
    """A magnitude with a time unit (``to``/``magnitude`` like pint)."""

    def __init__(self, magnitude, units="s"):
        if units not in _SECONDS:
            raise ValueError(f"unsupported unit {units!r}")
        self.magnitude = magnitude
        self.units = units

    def to(self, units):
        if units not in _SECONDS:
            raise ValueError(f"unsupported unit {units!r}")
        return Quantity(self.magnitude * _SECONDS[self.units] / _SECONDS[units], units)

    def __mul__(self, k):
        if isinstance(k, Quantity):
            raise TypeError("only scalar multiples of a time quantity are supported")
        return Quantity(self.magnitude * k, self.units)

    __rmul__ = __mul__

    def __truediv__(self, k):
        return Quantity(self.magnitude / k, self.units)

    def __eq__(self, other):
        return isinstance(other, Quantity) and self.to("s").magnitude == other.to("s").magnitude

    def __hash__(self):
        return hash(self.to("s").magnitude)

    def __repr__(self):
        return f"{self.magnitude} {self.units}"


s = Quantity(1.0, "s")
ms = Quantity(1.0, "ms")
us = Quantity(1.0, "us")
ns = Quantity(1.0, "ns")
minute = Quantity(1.0, "minute")
hour = Quantity(1.0, "hour")
