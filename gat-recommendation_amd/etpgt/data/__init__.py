"""Session batch layout, packing and the synthetic RetailRocket-shaped workload."""

from etpgt.data.batch import Caps, Data, SessionBatch, collate_sessions, pack_batch

__all__ = ["Caps", "Data", "SessionBatch", "collate_sessions", "pack_batch"]
