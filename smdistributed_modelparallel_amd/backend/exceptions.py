"""Exception hierarchy.

Mirrors the public exception names of the reference
(`smp/backend/exceptions.py:1-77`) so user code that catches them keeps working,
but the hierarchy is flattened into three families: configuration/argument
errors, runtime errors and unsupported-feature errors.
"""


class SMPError(Exception):
    """Base class of every error raised by the framework."""


# ---------------------------------------------------------------- validation
class SMPValidationError(SMPError):
    pass


class SMPInvalidArgumentError(SMPValidationError, ValueError):
    pass


class SMPConfigTypeError(SMPInvalidArgumentError, TypeError):
    """A config value has the wrong type (a TypeError, as in the reference)."""


class SMPConfigError(SMPValidationError):
    pass


class InvalidEnvironmentError(SMPValidationError):
    pass


class WorkerSizeError(SMPValidationError):
    pass


class NotInitializedError(SMPValidationError):
    def __init__(self, msg="smp.init() must be called before using this API."):
        super().__init__(msg)


# ------------------------------------------------------------------- runtime
class SMPRuntimeError(SMPError, RuntimeError):
    pass


class PipelineParallelBWDError(SMPRuntimeError):
    pass


class InvalidBwdCountError(PipelineParallelBWDError):
    pass


class StepFunctionCalledError(SMPRuntimeError):
    pass


class MissingOutputForModuleError(SMPRuntimeError):
    pass


class MissingPathFromComputationToLossError(SMPRuntimeError):
    pass


class DistributedModelNotWrappedError(SMPRuntimeError):
    pass


class CheckpointingError(SMPRuntimeError):
    pass


class PartitionError(SMPRuntimeError):
    pass


class TransportError(SMPRuntimeError):
    pass


class HIPExtensionMissingError(SMPRuntimeError):
    """Raised when a GPU op is requested but the in-tree HIP extension is not built."""


# --------------------------------------------------------------- unsupported
class SMPUnsupportedError(SMPError, NotImplementedError):
    pass


class UnsupportedCommunicationVolumeUnitError(SMPUnsupportedError):
    pass


class TracingEnd(Exception):
    """Internal control-flow signal: stop the step function once the traced forward ends
    (reference `patches/tracing.py:41-86`)."""
