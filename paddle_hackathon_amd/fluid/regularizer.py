from ..regularizer import L1Decay, L2Decay, L1DecayRegularizer, L2DecayRegularizer  # noqa: F401

__all__ = ["L1Decay", "L2Decay", "L1DecayRegularizer", "L2DecayRegularizer"]
