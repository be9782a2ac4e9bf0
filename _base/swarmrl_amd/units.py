"""
Minimal unit registry standing in for ``pint`` (absent from this image).

The reference converts every input to simulation units with pint
(swarmrl/engine/espresso.py:211-234: sim_length = 1 um, sim_time = 1 s,
sim_energy = 293 K * k_B, plus derived units).  This module provides the
subset of the pint API that the engine surface and its callers use:
``UnitRegistry().Quantity(value, "unit expr")``, ``ureg.define("a = expr")``,
``ureg.<unit>`` attributes, quantity arithmetic and ``.m_as("unit expr")``.
Unit expressions are products/quotients/powers of known names and numbers,
e.g. ``"pascal * second"``, ``"kg/meter**3"``, ``"sim_force/sim_velocity"``.
"""

from __future__ import annotations

import re
from typing import Dict, Tuple

import numpy as np

# dimension vector: (length, mass, time, temperature)
_DIMLESS = (0, 0, 0, 0)

_SI_UNITS: Dict[str, Tuple[float, Tuple[int, int, int, int]]] = {
    "meter": (1.0, (1, 0, 0, 0)),
    "metre": (1.0, (1, 0, 0, 0)),
    "m": (1.0, (1, 0, 0, 0)),
    "centimeter": (1e-2, (1, 0, 0, 0)),
    "millimeter": (1e-3, (1, 0, 0, 0)),
    "micrometer": (1e-6, (1, 0, 0, 0)),
    "micron": (1e-6, (1, 0, 0, 0)),
    "um": (1e-6, (1, 0, 0, 0)),
    "nanometer": (1e-9, (1, 0, 0, 0)),
    "nm": (1e-9, (1, 0, 0, 0)),
    "kilogram": (1.0, (0, 1, 0, 0)),
    "kg": (1.0, (0, 1, 0, 0)),
    "gram": (1e-3, (0, 1, 0, 0)),
    "g": (1e-3, (0, 1, 0, 0)),
    "second": (1.0, (0, 0, 1, 0)),
    "s": (1.0, (0, 0, 1, 0)),
    "millisecond": (1e-3, (0, 0, 1, 0)),
    "ms": (1e-3, (0, 0, 1, 0)),
    "microsecond": (1e-6, (0, 0, 1, 0)),
    "minute": (60.0, (0, 0, 1, 0)),
    "hour": (3600.0, (0, 0, 1, 0)),
    "kelvin": (1.0, (0, 0, 0, 1)),
    "K": (1.0, (0, 0, 0, 1)),
    "newton": (1.0, (1, 1, -2, 0)),
    "N": (1.0, (1, 1, -2, 0)),
    "joule": (1.0, (2, 1, -2, 0)),
    "J": (1.0, (2, 1, -2, 0)),
    "pascal": (1.0, (-1, 1, -2, 0)),
    "Pa": (1.0, (-1, 1, -2, 0)),
    "liter": (1e-3, (3, 0, 0, 0)),
    "radian": (1.0, _DIMLESS),
    "dimensionless": (1.0, _DIMLESS),
    # CODATA 2018 exact value (the one pint ships)
    "boltzmann_constant": (1.380649e-23, (2, 1, -2, -1)),
    "k_B": (1.380649e-23, (2, 1, -2, -1)),
}


def _dim_mul(a, b):
    return tuple(x + y for x, y in zip(a, b))


def _dim_div(a, b):
    return tuple(x - y for x, y in zip(a, b))


def _dim_pow(a, p):
    return tuple(int(x * p) for x in a)


class DimensionalityError(ValueError):
    pass


class Quantity:
    """A magnitude (float or ndarray) with an SI factor and a dimension."""

    __array_priority__ = 1000

    def __init__(self, registry, magnitude, factor: float, dims):
        self._reg = registry
        self.magnitude = magnitude
        self._factor = float(factor)
        self._dims = tuple(dims)

    # pint-compatible accessors
    @property
    def m(self):
        return self.magnitude

    @property
    def units(self):
        return (self._factor, self._dims)

    def _si(self):
        return np.asarray(self.magnitude, dtype=float) * self._factor

    def m_as(self, unit: str):
        factor, dims = self._reg._parse(unit)
        if dims != self._dims:
            raise DimensionalityError(
                f"cannot convert dimension {self._dims} to {dims} ({unit})"
            )
        val = np.asarray(self.magnitude, dtype=float) * (self._factor / factor)
        return float(val) if val.ndim == 0 else val

    def to(self, unit: str) -> "Quantity":
        factor, dims = self._reg._parse(unit)
        return Quantity(self._reg, self.m_as(unit), factor, dims)

    def _coerce(self, other):
        if isinstance(other, Quantity):
            return other
        return Quantity(self._reg, other, 1.0, _DIMLESS)

    def __mul__(self, other):
        o = self._coerce(other)
        return Quantity(
            self._reg,
            np.multiply(self.magnitude, o.magnitude),
            self._factor * o._factor,
            _dim_mul(self._dims, o._dims),
        )

    __rmul__ = __mul__

    def __truediv__(self, other):
        o = self._coerce(other)
        return Quantity(
            self._reg,
            np.divide(self.magnitude, o.magnitude),
            self._factor / o._factor,
            _dim_div(self._dims, o._dims),
        )

    def __rtruediv__(self, other):
        return self._coerce(other) / self

    def __pow__(self, p):
        return Quantity(
            self._reg,
            np.power(self.magnitude, p),
            self._factor**p,
            _dim_pow(self._dims, p),
        )

    def _same_dims(self, other):
        o = self._coerce(other)
        if o._dims != self._dims:
            raise DimensionalityError("incompatible dimensions")
        return o

    def __add__(self, other):
        o = self._same_dims(other)
        return Quantity(
            self._reg,
            np.add(self.magnitude, np.asarray(o.magnitude) * (o._factor / self._factor)),
            self._factor,
            self._dims,
        )

    __radd__ = __add__

    def __sub__(self, other):
        o = self._same_dims(other)
        return Quantity(
            self._reg,
            np.subtract(
                self.magnitude, np.asarray(o.magnitude) * (o._factor / self._factor)
            ),
            self._factor,
            self._dims,
        )

    def __rsub__(self, other):
        return self._coerce(other) - self

    def __neg__(self):
        return Quantity(self._reg, np.negative(self.magnitude), self._factor, self._dims)

    def _cmp_val(self, other):
        o = self._same_dims(other)
        return np.asarray(o.magnitude) * (o._factor / self._factor)

    def __lt__(self, other):
        return np.asarray(self.magnitude) < self._cmp_val(other)

    def __le__(self, other):
        return np.asarray(self.magnitude) <= self._cmp_val(other)

    def __gt__(self, other):
        return np.asarray(self.magnitude) > self._cmp_val(other)

    def __ge__(self, other):
        return np.asarray(self.magnitude) >= self._cmp_val(other)

    def __eq__(self, other):
        try:
            return np.asarray(self.magnitude) == self._cmp_val(other)
        except DimensionalityError:
            return False

    def __hash__(self):
        return id(self)

    def __len__(self):
        return len(self.magnitude)

    def __iter__(self):
        for v in np.asarray(self.magnitude):
            yield Quantity(self._reg, v, self._factor, self._dims)

    def __getitem__(self, key):
        return Quantity(
            self._reg, np.asarray(self.magnitude)[key], self._factor, self._dims
        )

    def __float__(self):
        if self._dims != _DIMLESS:
            raise DimensionalityError("only dimensionless quantities convert to float")
        return float(self.magnitude) * self._factor

    def __repr__(self):
        return f"<Quantity({self.magnitude}, SI factor {self._factor:g}, dims {self._dims})>"


_TOKEN = re.compile(r"\s*(\*\*|\*|/|\(|\)|[0-9.]+(?:[eE][-+]?\d+)?|[A-Za-z_][A-Za-z_0-9]*)")


class UnitRegistry:
    """Subset of ``pint.UnitRegistry`` used by the engine and its callers."""

    def __init__(self):
        self._units: Dict[str, Tuple[float, Tuple[int, int, int, int]]] = dict(_SI_UNITS)

    # ---- parsing
    def _parse(self, expr: str):
        if isinstance(expr, tuple):
            return expr
        tokens = [t for t in _TOKEN.findall(expr) if t]
        if "".join(tokens).replace(" ", "") != expr.replace(" ", ""):
            raise ValueError(f"cannot parse unit expression {expr!r}")
        self._tok = tokens
        self._pos = 0
        if not tokens:
            return 1.0, _DIMLESS
        val = self._expr()
        if self._pos != len(tokens):
            raise ValueError(f"cannot parse unit expression {expr!r}")
        return val

    def _peek(self):
        return self._tok[self._pos] if self._pos < len(self._tok) else None

    def _expr(self):
        f, d = self._power()
        while True:
            t = self._peek()
            if t == "*":
                self._pos += 1
                f2, d2 = self._power()
                f, d = f * f2, _dim_mul(d, d2)
            elif t == "/":
                self._pos += 1
                f2, d2 = self._power()
                f, d = f / f2, _dim_div(d, d2)
            elif t is not None and t not in (")",):
                # implicit multiplication ("293 kelvin")
                f2, d2 = self._power()
                f, d = f * f2, _dim_mul(d, d2)
            else:
                return f, d

    def _power(self):
        f, d = self._atom()
        if self._peek() == "**":
            self._pos += 1
            tok = self._peek()
            sign = 1
            if tok == "-":
                sign = -1
                self._pos += 1
                tok = self._peek()
            self._pos += 1
            p = sign * float(tok)
            f, d = f**p, _dim_pow(d, p)
        return f, d

    def _atom(self):
        t = self._peek()
        self._pos += 1
        if t == "(":
            v = self._expr()
            if self._peek() != ")":
                raise ValueError("unbalanced parenthesis in unit expression")
            self._pos += 1
            return v
        if t is not None and re.match(r"^[0-9.]", t):
            return float(t), _DIMLESS
        if t in self._units:
            return self._units[t]
        raise ValueError(f"unknown unit {t!r}")

    # ---- public API
    def define(self, definition: str) -> None:
        name, expr = (s.strip() for s in definition.split("=", 1))
        self._units[name] = self._parse(expr)

    def Quantity(self, value, unit: str = "dimensionless") -> Quantity:  # noqa: N802
        factor, dims = self._parse(unit)
        if isinstance(value, (list, tuple)):
            value = np.asarray(value, dtype=float)
        return Quantity(self, value, factor, dims)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self._units:
            f, d = self._units[name]
            return Quantity(self, 1.0, f, d)
        raise AttributeError(name)


def ensure_quantity_array(values, ureg: UnitRegistry) -> Quantity:
    """convert_array_of_pint_to_pint_of_array (utils.py:460-468)."""
    first = values[0]
    unit = (first._factor, first._dims)
    mags = [v.m_as(unit) for v in values]
    return Quantity(ureg, np.asarray(mags), first._factor, first._dims)
