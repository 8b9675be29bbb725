"""Footstep sequence: the input producer of the CoP bounds.

Behaviour of the reference ``generators/footstep_generator.py:7-49`` (restated, not copied):
two standing feet at x = 0, then alternating steps of ``step_length`` until ``distance`` is
covered (the last one at most half a step), then the trailing foot joins the leading one.
Each contact is a 0.11 m × 0.05 m rectangle (``footstep_generator.py:34``).
"""

from typing import List, Tuple

FOOT_SHAPE = (0.11, 0.05)  # length (x) × width (y), footstep_generator.py:34
FRICTION = 0.7


class Contact:
    """A rectangular foot contact centred on (x, y) with its CoP box ``z_min``/``z_max``."""

    def __init__(self, x: float, y: float, shape: Tuple[float, float], friction: float):
        self.x, self.y = x, y
        self.shape, self.friction = shape, friction
        half_l, half_w = shape[0] / 2, shape[1] / 2
        self.z_max = [x + half_l, y + half_w]
        self.z_min = [x - half_l, y - half_w]


def _advance(x: float, distance: float, step_length: float) -> float:
    remaining = distance - x
    if remaining <= step_length:
        return x + min(remaining, 0.5 * step_length)
    return x + step_length


def generate_footsteps(distance: float, step_length: float, foot_spread: float) -> List[Contact]:
    """Footstep list for a straight walk of ``distance`` metres."""
    feet = [Contact(0., -foot_spread, FOOT_SHAPE, FRICTION),
            Contact(0., +foot_spread, FOOT_SHAPE, FRICTION)]
    x, side = 0., foot_spread
    while x < distance:
        x = _advance(x, distance, step_length)
        side = -side
        feet.append(Contact(x, side, FOOT_SHAPE, FRICTION))
    feet.append(Contact(x, -side, FOOT_SHAPE, FRICTION))
    return feet
