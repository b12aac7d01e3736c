"""Reference-compatible API surface (hiropppe/RocAlphaGo module paths).

Every module here re-exports the MI355X-native implementation in ``rocalphago_amd``.
"""
