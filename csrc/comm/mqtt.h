// Minimal MQTT 3.1.1 client and broker (native, no paho / mosquitto).
//
// The reference's mqttsink / mqttsrc ride on paho-mqtt-c against an external
// broker (gst/mqtt/mqttsink.c:751-875, mqttsrc.c:1254-1340), and the
// "HYBRID" connect-type of nnstreamer-edge uses an MQTT broker only to
// discover the TCP data endpoint.  Neither library exists here, so nnsx
// speaks the protocol itself: CONNECT / PUBLISH (QoS 0 and 1, retain) /
// SUBSCRIBE (+ and # wildcards) / PINGREQ / DISCONNECT.  MqttBroker is a
// small in-process broker (retained messages, wildcard fan-out) so pipelines
// and tests work without an external one.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace nnsx {
namespace comm {

struct MqttMessage {
  std::string topic;
  std::string payload;
  int qos = 0;
  bool retain = false;
};

bool mqtt_topic_matches(const std::string& filter, const std::string& topic);

class MqttClient {
 public:
  ~MqttClient();
  // keepalive_s = 0 disables PINGREQ
  bool connect(const std::string& host, int port, const std::string& client_id, int keepalive_s, bool clean_session,
               int timeout_ms, std::string* err);
  bool publish(const std::string& topic, const void* data, size_t len, int qos, bool retain, int timeout_ms = 5000);
  // publish header + body without concatenating them first
  bool publish2(const std::string& topic, const void* hdr, size_t hlen, const void* body, size_t blen, int qos,
                bool retain, int timeout_ms = 5000);
  bool subscribe(const std::string& filter, int qos, int timeout_ms = 5000);
  // pop one received PUBLISH; false on timeout (*timed_out) or lost connection
  bool recv(MqttMessage* m, int timeout_ms, bool* timed_out = nullptr);
  void close();  // DISCONNECT + join
  bool connected() const { return alive_.load(); }

 private:
  bool send_packet(uint8_t type_flags, const std::string& var, const void* p1, size_t n1, const void* p2, size_t n2);
  bool wait_ack(uint16_t id, int timeout_ms);
  void reader();
  void pinger(int keepalive_s);

  int fd_ = -1;
  std::atomic<bool> alive_{false};
  std::mutex wmu_;  // socket writes
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<MqttMessage> inbox_;
  std::map<uint16_t, bool> acks_;
  uint16_t next_id_ = 1;
  std::thread reader_, pinger_;
  std::atomic<bool> stop_{false};
};

class MqttBroker {
 public:
  ~MqttBroker() { stop(); }
  bool start(const std::string& host, int port, std::string* err);  // port 0: ephemeral
  void stop();
  int port() const { return port_; }
  size_t clients();
  uint64_t messages() const { return published_.load(); }

 private:
  struct Client;
  void accept_loop();
  void serve(std::shared_ptr<Client> c);
  void route(const MqttMessage& m);

  int lfd_ = -1, port_ = 0;
  std::atomic<bool> running_{false};
  std::thread acc_;
  std::mutex mu_;
  std::vector<std::shared_ptr<Client>> clients_;
  std::vector<std::thread> workers_;
  std::map<std::string, MqttMessage> retained_;
  std::atomic<uint64_t> published_{0};
};

// Process-wide brokers by port (the `nns.MqttBroker` / nnsx-launch helper).
std::shared_ptr<MqttBroker> mqtt_broker_start(const std::string& host, int port, std::string* err);

}  // namespace comm
}  // namespace nnsx
