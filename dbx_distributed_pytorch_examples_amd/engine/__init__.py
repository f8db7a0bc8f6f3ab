"""Execution engines: the graph-captured native ResNet program and the generic autograd path."""
