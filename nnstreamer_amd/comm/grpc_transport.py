"""gRPC endpoint for tensor_src_grpc / tensor_sink_grpc (csrc/comm/grpc_bridge.h).

The reference's TensorService (ext/nnstreamer/include/nnstreamer.proto):

    service TensorService {
      rpc SendTensors (stream Tensors) returns (google.protobuf.Empty);  // client -> server
      rpc RecvTensors (google.protobuf.Empty) returns (stream Tensors);  // server -> client
    }

served / called with grpcio generic handlers on raw bytes: the `Tensors`
messages are serialized natively (protobuf or flatbuf IDL), and
google.protobuf.Empty is the empty byte string.  Roles (reference defaults:
sink = client, source = server):

    sink + client   SendTensors caller, one request stream for the run
    sink + server   RecvTensors server, every subscribed call gets each buffer
    src  + server   SendTensors server, requests from any client are queued
    src  + client   RecvTensors caller, the response stream feeds the queue
"""
from __future__ import annotations

import queue
import threading
from concurrent import futures

import grpc


def _ident(b):
    return b


_END = object()


class Endpoint:
    def __init__(self, server: bool, sending: bool, idl: str, host: str, port: int, blocking: bool):
        self.server, self.sending, self.blocking = server, sending, blocking
        self.service = f"nnstreamer.{idl.lower()}.TensorService"
        self.target = f"{host or 'localhost'}:{port}"
        self._port = port
        self._q: "queue.Queue" = queue.Queue(maxsize=64)  # received messages (source side)
        self._subs = []  # server sink: per-call queues
        self._lock = threading.Lock()
        self._stopped = threading.Event()
        self._srv = self._ch = self._fut = self._outq = None

    # ----------------------------------------------------------- lifecycle ----
    def start(self) -> str:
        try:
            if self.server:
                self._srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
                handlers = {
                    "SendTensors": grpc.stream_unary_rpc_method_handler(
                        self._serve_send, request_deserializer=_ident, response_serializer=_ident),
                    "RecvTensors": grpc.unary_stream_rpc_method_handler(
                        self._serve_recv, request_deserializer=_ident, response_serializer=_ident),
                }
                self._srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(self.service, handlers),))
                self._port = self._srv.add_insecure_port(self.target)
                if not self._port:
                    return f"cannot bind {self.target}"
                self._srv.start()
                return ""
            self._ch = grpc.insecure_channel(self.target)
            grpc.channel_ready_future(self._ch).result(timeout=10)
            if self.sending:
                self._outq = queue.Queue()
                call = self._ch.stream_unary(f"/{self.service}/SendTensors", request_serializer=_ident,
                                             response_deserializer=_ident)
                self._fut = call.future(self._requests())
            else:
                call = self._ch.unary_stream(f"/{self.service}/RecvTensors", request_serializer=_ident,
                                             response_deserializer=_ident)
                stream = call(b"")
                threading.Thread(target=self._pump, args=(stream,), daemon=True).start()
            return ""
        except grpc.FutureTimeoutError:
            return f"cannot connect to {self.target}"
        except Exception as e:  # noqa: BLE001
            return str(e)

    def stop(self) -> None:
        if self._stopped.is_set():
            return
        self._stopped.set()
        with self._lock:
            for q in self._subs:
                q.put(_END)
        if self._outq is not None:
            self._outq.put(_END)
            try:
                self._fut.result(timeout=10)
            except Exception:  # noqa: BLE001
                pass
        if self._srv is not None:
            self._srv.stop(grace=1.0)
        if self._ch is not None:
            self._ch.close()

    def port(self) -> int:
        return int(self._port)

    # ------------------------------------------------------------ sink side ----
    def send(self, msg: bytes) -> bool:
        if self._stopped.is_set():
            return False
        if self.server:
            with self._lock:
                for q in self._subs:
                    q.put(msg)
            return True
        self._outq.put(msg)
        return not self._fut.done() or self._fut.exception() is None

    def _requests(self):
        while True:
            m = self._outq.get()
            if m is _END:
                return
            yield m

    def _serve_recv(self, request, context):
        q: "queue.Queue" = queue.Queue()
        with self._lock:
            self._subs.append(q)
        try:
            while context.is_active():
                try:
                    m = q.get(timeout=0.1)
                except queue.Empty:
                    continue
                if m is _END:
                    return
                yield m
        finally:
            with self._lock:
                self._subs.remove(q)

    def subscribers(self) -> int:
        with self._lock:
            return len(self._subs)

    # ---------------------------------------------------------- source side ----
    def recv(self, timeout_ms: int):
        try:
            m = self._q.get(timeout=max(0, timeout_ms) / 1000.0)
        except queue.Empty:
            return (-1, b"") if self._stopped.is_set() else (0, b"")
        if m is _END:
            return (-1, b"")
        return (1, m)

    def _serve_send(self, request_iterator, context):
        for m in request_iterator:
            if self._stopped.is_set():
                break
            self._q.put(m)
        return b""

    def _pump(self, stream):
        try:
            for m in stream:
                self._q.put(m)
        except grpc.RpcError:
            pass
        self._q.put(_END)
