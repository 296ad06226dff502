"""Grid (reference: abmarl/sim/gridworld/grid.py:7-143).

Two uses:
  * the fused step programs never touch it: each step kernel rebuilds a
    per-env occupancy table in LDS from the lanes' positions, and the in-cell
    insertion order of the reference's dict cells is carried by a per-agent
    placement sequence number (seq);
  * the component plugin API (components.py, component_runtime.py) keeps it
    as the reference's container: cells are insertion-ordered dicts
    (agent id -> agent), mirrored from the engine after every component
    operation, and ``query`` / ``place`` / ``remove`` / ``reset`` /
    ``grid[r, c]`` behave as the reference's for user code that edits it.
"""
import copy

import numpy as np

from abmarl_amd.sim import host_version


class Grid:
    def __init__(self, rows, cols, overlapping=None, **kwargs):
        assert type(rows) is int and rows > 0, "Rows must be a positive integer."
        assert type(cols) is int and cols > 0, "Cols must be a positive integer."
        self._internal = np.empty((rows, cols), dtype=object)
        self.overlapping = overlapping

    @property
    def rows(self):
        return self._internal.shape[0]

    @property
    def cols(self):
        return self._internal.shape[1]

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

    # ----------------------------------------------- container (grid.py:73-143)
    def reset(self, **kwargs):
        """Every cell an empty dict (grid.py:73-79)."""
        for i in range(self.rows):
            for j in range(self.cols):
                self._internal[i, j] = {}
        host_version.bump()

    def query(self, agent, ndx):
        """The cell is empty, or every occupant's encoding may overlap this
        agent's (a missing overlapping key means False, grid.py:81-105)."""
        ndx = tuple(ndx)
        if self._internal[ndx]:
            try:
                return all(other.encoding in self.overlapping[agent.encoding]
                           for other in self._internal[ndx].values())
            except KeyError:
                return False
        return True

    def place(self, agent, ndx):
        """Append the agent to the cell if query allows it (grid.py:107-129)."""
        ndx = tuple(ndx)
        if self.query(agent, ndx):
            self._internal[ndx][agent.id] = agent
            agent.position = np.array(ndx)
            host_version.bump()
            return True
        return False

    def remove(self, agent, ndx):
        """grid.py:131-140 (KeyError if the agent is not in the cell)."""
        del self._internal[tuple(ndx)][agent.id]
        host_version.bump()

    def __getitem__(self, subscript):
        return self._internal.__getitem__(subscript)
