"""libgtr_hip binding (ctypes), engine and autograd ops."""
