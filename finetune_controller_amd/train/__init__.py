"""Worker runtime: training loop, data, optimizer (the PyTorchJob container's entry point)."""
