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


class DDPNotEnabledError(SMPValidationError):
    """A torch.distributed process group was requested but none exists (reference
    `torch/exceptions.py:24-27`)."""

    def __str__(self):
        return "torch.distributed is not initialized for this group: enable ddp in the smp config"


class InvalidCommGroupError(SMPValidationError):
    """A barrier / collective was given something that is not a CommGroup (reference
    `torch/exceptions.py:29-35`)."""

    def __init__(self, group):
        super().__init__(group)
        self.group = group

    def __str__(self):
        return f"invalid communication group {self.group!r}: expected a smp.CommGroup"


class DistTransformerConfigError(SMPInvalidArgumentError):
    """An smp.nn transformer module was given an unsupported combination of options
    (reference `torch/exceptions.py:53`)."""


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


class MissingPathFromComputationToModuleOutputError(SMPRuntimeError):
    """A remote module's output has no autograd path to the outputs of the module that
    called it (reference `torch/exceptions.py:527-541`)."""

    def __init__(self, parent_module_name, module_name):
        super().__init__(parent_module_name, module_name)
        self.parent_module_name = parent_module_name
        self.module_name = module_name

    def __str__(self):
        return (f"during execution of {self.parent_module_name!r}: the output of module {self.module_name!r} has no "
                "path to the outputs backward is called on; use it, detach it, or set "
                "SMP_SKIP_GRAPH_VALIDATION=1 (the pipeline engine then runs the graph, the unused output gets no "
                "gradient)")


class MissingPathFromModuleInputToModuleOutputError(SMPRuntimeError):
    """An input of a pipeline-executed module requires grad but does not reach the
    module's outputs (reference `torch/exceptions.py:543-556`)."""

    def __init__(self, module_name, idx):
        super().__init__(module_name, idx)
        self.module_name = module_name
        self.idx = idx

    def __str__(self):
        return (f"during execution of {self.module_name!r}: input tensor #{self.idx} requires grad but has no path "
                "to the module outputs; detach it, or set SMP_SKIP_GRAPH_VALIDATION=1 (the input then gets no "
                "gradient)")


class NotSupportedByFastModeError(SMPRuntimeError):
    """Reference `smp/torch/exceptions.py:355-362`: the model cannot run in fast mode (the
    parent used a tensor that was transmitted child-to-child), or its graph changed after
    the direct-consumer maps were recorded."""

    def __init__(self, graph_change=False, detail=""):
        self.graph_change = graph_change
        msg = ("A change in model graph is detected. Graph changes are not supported in fast mode, please set "
               "'fast_mode' to False." if graph_change else
               "Model is not supported by fast mode, please set 'fast_mode' to False.")
        super().__init__(msg + (f" ({detail})" if detail else ""))


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


# ------------------------------------------------------- HuggingFace translation
class HFConfigError(SMPValidationError, NotImplementedError):
    """An HF model config or forward argument the DistributedTransformer translation cannot
    reproduce (reference `torch/exceptions.py:57-82`: one class per model family)."""


class HFBertConfigError(HFConfigError):
    pass


class HFRobertaConfigError(HFConfigError):
    pass


class HFGPT2ConfigError(HFConfigError):
    pass


class HFGPTJConfigError(HFConfigError):
    pass


class HFGPTNeoConfigError(HFConfigError):
    pass


class HFGPTNeoxConfigError(HFConfigError):
    pass


class HFT5ConfigError(HFConfigError):
    pass


class HFViTConfigError(HFConfigError):
    pass


# ------------------------------------------------- reference exception names
# Every exception class the reference defines (`backend/exceptions.py`, `torch/exceptions.py`)
# exists here under its name, placed in this hierarchy, so user code catching them keeps
# working; the ones this framework raises for the same condition are raised under these names
# (split, step outputs, checkpoints, a second DistributedModel).
class CommGroupConfigError(SMPValidationError):
    pass


class LoggingConfigError(SMPValidationError):
    pass


class InvalidTransactionIDError(SMPValidationError):
    pass


class InvalidLinkIDError(SMPValidationError):
    pass


class InvalidStepOutputError(SMPInvalidArgumentError):
    """A StepOutput was built from something other than a list / tuple, or reduced over
    non-tensor outputs."""


class TensorSplitError(SMPRuntimeError, SMPInvalidArgumentError):
    """A step input cannot be split into the configured number of microbatches."""


class InitializationError(SMPRuntimeError):
    pass


class SMPSegFault(SMPRuntimeError):
    pass


class DDPConfigError(SMPValidationError):
    pass


class HorovodConfigError(SMPValidationError):
    pass


class CheckpointingConfigError(SMPValidationError):
    pass


class DistEmbeddingConfigError(SMPValidationError):
    pass


class ModelTooSmallError(SMPValidationError):
    pass


class InvalidSeqLenPrescaledBatchError(SMPValidationError):
    pass


class MemoryWeightError(SMPValidationError):
    pass


class CostListError(SMPValidationError):
    pass


class MultipleDistributedModelError(SMPValidationError, SMPRuntimeError):
    """More than one smp.DistributedModel in a process."""


class BwdExecutionNotInStepFnError(SMPValidationError):
    pass


class FwdExecutionNotInStepFnError(SMPValidationError):
    pass


class ModelNotPartitionedError(SMPValidationError):
    pass


class HiddenDimError(SMPValidationError):
    pass


class SplitShapeLenError(SMPValidationError):
    pass


class SplitShapeMismatchError(SMPValidationError):
    pass


class ShiftValueError(SMPValidationError):
    pass


class PaddingSizeError(SMPValidationError):
    pass


class DistributedModelWrappedError(SMPValidationError):
    pass


class InvalidPartitionIDError(SMPValidationError):
    pass


class HFNotAvailableError(SMPValidationError):
    pass


class SMPCheckpointError(CheckpointingError, SMPValidationError):
    """Base of the checkpoint-content errors (a CheckpointingError too)."""


class MissingCheckpointFilesError(SMPCheckpointError):
    pass


class IncompatibleCheckpointRankFoundError(SMPCheckpointError):
    pass


class IncompatibleCheckpointFoundError(SMPCheckpointError):
    pass


class MissingKeysInCheckpointError(SMPCheckpointError):
    pass


class RemoteBufferShouldNotExistError(SMPCheckpointError):
    pass


class RemoteBufferShouldExistError(SMPCheckpointError):
    pass


class InvalidReturnTypeFromCheckpointedModuleError(SMPCheckpointError):
    pass


class FusedLAMBError(SMPUnsupportedError):
    pass


class DelayedParamDeviceError(SMPUnsupportedError):
    pass


class UnsupportedTorchVersionError(SMPUnsupportedError):
    pass


class UnsupportedReducerTypeError(SMPUnsupportedError):
    pass


class UnsupportedTPModuleError(SMPUnsupportedError):
    pass


class TPModuleRegisterError(SMPUnsupportedError):
    pass


class MultipleDtypeOptShardingError(SMPUnsupportedError):
    pass


class SequentialBackwardBrokenError(SMPUnsupportedError):
    pass


class RecursionDepthExceededDuringSerializationError(SMPUnsupportedError):
    pass


class UnsupportedMessageError(SMPUnsupportedError):
    pass


class UnsupportedShardedConfigError(SMPUnsupportedError, RuntimeError):
    pass


class ScaledBatchBufNotInDistModuleError(SMPRuntimeError):
    pass


class InvalidHandleError(SMPRuntimeError):
    pass


class MissingParentModuleError(SMPRuntimeError):
    pass


class MissingModuleError(SMPRuntimeError):
    pass


class ParentNodeExistingError(SMPRuntimeError):
    pass


class ChildNodeExistingError(SMPRuntimeError):
    pass


class UnrecognizedHFKeyError(SMPRuntimeError):
    pass


class CustomSoftmaxKernelDtypeError(SMPRuntimeError):
    pass


class MissingGradientError(SMPRuntimeError):
    pass


class GradRequireGradError(SMPRuntimeError):
    pass


class SMPAMPError(SMPRuntimeError):
    pass


class InvalidRequestError(SMPRuntimeError):
    pass


class InvalidExecutorError(SMPRuntimeError):
    pass


class NonDummyTensorError(SMPRuntimeError):
    pass


class InvalidParentModuleError(SMPRuntimeError):
    pass


class NumParametersNotMatchError(SMPRuntimeError):
    pass


class TracingEnd(Exception):
    """Internal control-flow signal: stop the step function once the traced forward ends
    (reference `patches/tracing.py:41-86`)."""
