"""A counter of host-side edits to simulation state: agent position /
health / active and the Grid's cells (grid.py place / remove / reset).  The
component runtime (sim/gridworld/component_runtime.py) reads it to skip
re-uploading state the device already holds; code that edits state in
place (a cell dict, a position array) without these setters is not seen."""
VERSION = [0]


def bump():
    VERSION[0] += 1
