"""Placement core: exact subset search, Gaia tree policies, reference (legacy) formulas."""
from .core import (NoFeasiblePlacement, Placement, PlacementPolicy, Problem, evaluate, place_fraction, score_from_objective, select,
                   worst)
from .gaia import CostTree, TreeNode, fragment, gaia_schedule, link, singular, tree_from_spec, tree_from_topology
from .legacy import design_farthest_single, design_greedy_select, legacy_score, legacy_score_of_set
from .defrag import DefragPlan, Move, plan_defrag

__all__ = [
    "NoFeasiblePlacement", "Placement", "PlacementPolicy", "Problem", "evaluate", "place_fraction", "score_from_objective", "select",
    "worst",
    "CostTree", "TreeNode", "fragment", "gaia_schedule", "link", "singular", "tree_from_spec", "tree_from_topology",
    "design_farthest_single", "design_greedy_select", "legacy_score", "legacy_score_of_set",
    "DefragPlan", "Move", "plan_defrag",
]
