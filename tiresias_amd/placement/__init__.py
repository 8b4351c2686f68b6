from .schemes import PLACEMENTS, Placement, make_placement

__all__ = ["PLACEMENTS", "Placement", "make_placement"]
