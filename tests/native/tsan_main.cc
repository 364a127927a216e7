// Host-runtime race check (SURVEY.md §5 "race detection"): a ThreadSanitizer
// build of the native runtime (no libtorch / Python) drives the threaded
// parts -- queue / tee threads, collect-pads muxing, the query server and
// client, pub/sub, rank groups over the TCP store, the MQTT broker -- and
// TSan reports any data race (exit code 66).  Built and run by
// scripts/tsan_check.sh.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "comm/mqtt.h"
#include "runtime/pipeline.h"

using namespace nnsx;

namespace {

int failures = 0;

void run(const std::string& desc, int64_t timeout_ms = 30000) {
  auto p = parse_launch(desc);
  std::string err;
  const bool ok = p->run_until_eos(timeout_ms * 1000000, &err);
  p->set_state(State::NULL_);
  std::printf("%s  %s%s\n", ok ? "ok  " : "FAIL", desc.substr(0, 90).c_str(), ok ? "" : ("  (" + err + ")").c_str());
  if (!ok) ++failures;
}

}  // namespace

int main() {
  const std::string src = "videotestsrc num-buffers=200 ! video/x-raw,format=RGB,width=32,height=32,framerate=0/1 "
                          "! tensor_converter";
  // thread boundaries and fan-out / fan-in
  run(src + " ! queue ! tensor_transform mode=arithmetic option=typecast:float32,mul:2 ! queue ! fakesink");
  run(src + " ! tee name=t t. ! queue ! tensor_mux name=m sync-mode=nosync ! fakesink "
            "t. ! queue ! tensor_transform mode=typecast option=float32 ! m.");
  run(src + " ! tensor_aggregator frames-out=4 frames-dim=3 ! queue ! tensor_demux name=d d.src_0 ! queue ! fakesink");
  // sparse codec round trip, protobuf serialisation round trip, tensor_if
  run(src + " ! tensor_sparse_enc ! queue ! tensor_sparse_dec ! fakesink");
  run(src + " ! tensor_decoder mode=protobuf ! queue ! tensor_converter ! fakesink");
  run(src + " ! tensor_if name=tif compared-value=TENSOR_AVERAGE_VALUE supplied-value=100 operator=GT "
            "then=PASSTHROUGH else=PASSTHROUGH tif.src_0 ! queue ! fakesink tif.src_1 ! queue ! fakesink");
  // native gRPC (HTTP/2): source server thread + sink client pipeline
  {
    auto server = parse_launch("tensor_src_grpc name=gs server=true port=0 ! other/tensors,format=static,"
                               "num_tensors=1,dimensions=3:32:32:1,types=uint8,framerate=30/1 ! queue ! fakesink");
    server->set_state(State::PLAYING);
    std::string port = "0";
    for (int i = 0; i < 500 && port == "0"; ++i) {
      port = server->get_by_name("gs")->get_property("port");
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    run(src + " ! tensor_sink_grpc host=127.0.0.1 port=" + port);
    server->set_state(State::NULL_);
  }
  // tensor_query in-process over TCP: server thread + client pipeline
  {
    auto server = parse_launch(
        "tensor_query_serversrc name=qs port=0 id=5 ! other/tensors,format=static,num_tensors=1,"
        "dimensions=3:32:32:1,types=uint8,framerate=0/1 ! queue ! tensor_query_serversink id=5");
    server->set_state(State::PLAYING);
    std::string port = "0";
    for (int i = 0; i < 500 && port == "0"; ++i) {
      port = server->get_by_name("qs")->get_property("port");
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    std::vector<std::thread> clients;
    for (int c = 0; c < 2; ++c)
      clients.emplace_back([&] { run(src + " ! tensor_query_client dest-port=" + port + " max-request=2 ! fakesink"); });
    for (auto& t : clients) t.join();
    server->set_state(State::NULL_);
  }
  // MQTT broker + pub/sub (broker threads, client reader / pinger threads)
  {
    std::string err;
    auto broker = comm::mqtt_broker_start("127.0.0.1", 0, &err);
    const std::string bp = std::to_string(broker->port());
    std::thread sub([&] { run("mqttsrc port=" + bp + " sub-topic=tsan sub-timeout=1000000 ! fakesink", 60000); });
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    run(src + " ! mqttsink port=" + bp + " pub-topic=tsan");
    sub.join();
    broker->stop();
  }
  // rank groups: three "ranks" in one process over the TCP store
  {
    const std::string store = "127.0.0.1:" + std::to_string(39000 + (std::rand() % 2000));
    std::vector<std::thread> ranks;
    for (int r = 0; r < 3; ++r)
      ranks.emplace_back([&, r] {
        run(src + " ! tensor_allgather comm-backend=tcp world-size=3 rank=" + std::to_string(r) + " store=" + store +
            " ! fakesink");
      });
    for (auto& t : ranks) t.join();
  }
  std::printf("%d failure(s)\n", failures);
  return failures ? 1 : 0;
}
