"""Session batch layout, packing and the synthetic RetailRocket-shaped workload."""

from etpgt.data.batch import Caps, SessionBatch, collate_sessions, pack_batch

__all__ = ["Caps", "SessionBatch", "collate_sessions", "pack_batch"]
