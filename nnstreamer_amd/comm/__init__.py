"""Transports driven from Python: the grpcio runtime behind tensor_src_grpc /
tensor_sink_grpc (see csrc/comm/grpc_bridge.h)."""
