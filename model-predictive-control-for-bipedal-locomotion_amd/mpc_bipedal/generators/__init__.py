"""Generators for footsteps and CoP bounds (the solver's input producer)."""

from .footstep_generator import Contact, generate_footsteps
from .cop_generator import CoPGenerator, State

__all__ = ['Contact', 'generate_footsteps', 'CoPGenerator', 'State']
