"""CDNA4 HIP kernel wrappers (GPU) with PyTorch reference math for CPU tensors."""
