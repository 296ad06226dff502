"""Grid description (reference: abmarl/sim/gridworld/grid.py:7-71).

On the engine the grid is not stored at all: each step kernel rebuilds a
per-env occupancy table in LDS from the agents' positions (count + XOR of
encodings per cell), and the in-cell insertion order of the reference's
dict cells is carried by a per-agent placement sequence number.  This
class keeps the host-side facts: shape and the (symmetrised) overlap map.
"""
import copy


class Grid:
    def __init__(self, rows, cols, overlapping=None, **kwargs):
        assert type(rows) is int and rows > 0, "Rows must be a positive integer."
        assert type(cols) is int and cols > 0, "Cols must be a positive integer."
        self._rows = rows
        self._cols = cols
        self.overlapping = overlapping

    @property
    def rows(self):
        return self._rows

    @property
    def cols(self):
        return self._cols

    @property
    def overlapping(self):
        return self._overlapping

    @overlapping.setter
    def overlapping(self, value):
        """Force symmetry: if a may overlap b then b may overlap a (grid.py:53-71)."""
        if value is None:
            self._overlapping = {}
            return
        assert type(value) is dict, "Overlaping must be dictionary."
        sym = copy.deepcopy(value)
        for enc, others in value.items():
            assert type(enc) is int, "All keys in overlapping dict must be integers."
            assert type(others) is set, "All values in overlapping dict must be sets."
            for other in others:
                assert type(other) is int, \
                    "All elements in overlapping dict values must be integers."
                sym.setdefault(other, set()).add(enc)
        self._overlapping = sym

    def overlap_bits(self):
        """encoding -> bitmask of encodings it may share a cell with."""
        bits = {}
        for enc, others in self._overlapping.items():
            for o in others:
                bits[enc] = bits.get(enc, 0) | (1 << o)
        return bits
