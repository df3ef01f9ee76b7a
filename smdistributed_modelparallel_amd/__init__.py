"""smdistributed_modelparallel_amd: MI355X-native pipeline / tensor / data parallel
training library with the smdistributed.modelparallel API.

    import smdistributed_modelparallel_amd.torch as smp
"""
__version__ = "0.1.0"
