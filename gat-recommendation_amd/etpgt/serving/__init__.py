"""Single-session serving on the HIP path."""

from etpgt.serving.recommender import Recommender, ValidatedRequest

__all__ = ["Recommender", "ValidatedRequest"]
