// mqttsink / mqttsrc: publish / subscribe tensor (or any) buffers through an
// MQTT broker, wire-compatible with the reference elements.
//
// Reference: gst/mqtt/mqttcommon.h:29-63 (1024-byte GstMQTTMessageHdr before
// the concatenated memories), mqttsink.c (props :67-89, header fill
// :691-715, render :751-875), mqttsrc.c (props :60-75 / :255-270, create
// :722-815 -- sub-timeout ends the stream, timestamps re-based by the
// publisher/subscriber base-time epochs :1380-1410), ntputil.c (optional
// NTP epoch).  The MQTT protocol is spoken natively (comm/mqtt.h); paho is
// not needed.
#include <netdb.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <atomic>
#include <cstring>

#include "comm/mqtt.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

constexpr size_t kHdrLen = 1024;
constexpr size_t kMaxMems = 16;
constexpr size_t kCapsLen = 512;
constexpr uint64_t kNone = ~0ull;  // GST_CLOCK_TIME_NONE

// GstMQTTMessageHdr on LP64 hosts (guint + pad, gsize[16], 2 x gint64, 3 x GstClockTime, gchar[512])
struct MqttHdr {
  uint32_t num_mems;
  uint32_t pad_;
  uint64_t size_mems[kMaxMems];
  int64_t base_time_epoch;
  int64_t sent_time_epoch;
  uint64_t duration, dts, pts;
  char caps[kCapsLen];
  uint8_t reserved[kHdrLen - 176 - kCapsLen];
};
static_assert(sizeof(MqttHdr) == kHdrLen, "mqtt header must be 1024 bytes");
static_assert(offsetof(MqttHdr, caps) == 176, "mqtt header layout");

std::atomic<unsigned> g_mqtt_seq{0};

std::string default_client_id(const char* role) {
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  return strfmt(host, "_", getpid(), "_", role, g_mqtt_seq++);
}

// SNTP: offset (ns) to add to the local epoch; 0 when no server answers.
// (ntputil.c:106-245 -- the reference averages nothing either: first answer wins)
int64_t ntp_offset_ns(const std::string& servers) {
  for (auto& entry : split(servers, ',')) {
    const std::string e = strip(entry);
    if (e.empty()) continue;
    std::string host = e;
    std::string port = "123";
    const size_t c = e.rfind(':');
    if (c != std::string::npos) {
      host = e.substr(0, c);
      port = e.substr(c + 1);
    }
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_DGRAM;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) continue;
    const int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd < 0) {
      freeaddrinfo(res);
      continue;
    }
    timeval tv{1, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    uint8_t pkt[48] = {0x1b};  // LI 0, VN 3, mode 3 (client)
    const int64_t t0 = epoch_ns();
    int64_t off = 0;
    bool ok = false;
    if (::sendto(fd, pkt, sizeof(pkt), 0, res->ai_addr, res->ai_addrlen) == sizeof(pkt) &&
        ::recv(fd, pkt, sizeof(pkt), 0) == sizeof(pkt)) {
      const int64_t t1 = epoch_ns();
      const uint32_t sec = (uint32_t(pkt[40]) << 24) | (uint32_t(pkt[41]) << 16) | (uint32_t(pkt[42]) << 8) | pkt[43];
      const uint32_t frac = (uint32_t(pkt[44]) << 24) | (uint32_t(pkt[45]) << 16) | (uint32_t(pkt[46]) << 8) | pkt[47];
      const int64_t server = (static_cast<int64_t>(sec) - 2208988800LL) * 1000000000LL +
                             static_cast<int64_t>((static_cast<uint64_t>(frac) * 1000000000ULL) >> 32);
      off = server - (t0 + (t1 - t0) / 2);
      ok = true;
    }
    ::close(fd);
    freeaddrinfo(res);
    if (ok) return off;
  }
  return 0;
}

// ============================================================== mqttsink ====
class MqttSink : public BaseSink {
 public:
  explicit MqttSink(const std::string& name) : BaseSink("mqttsink", name, Caps::Any()) {
    prop_bool("debug", &debug_, "Produce extra verbose output for debug purpose");
    prop_string("client-id", &client_id_, "The client identifier passed to the server (broker)");
    prop_string("host", &host_, "Host (broker) to connect to");
    prop_string("port", &port_, "Network port of host (broker) to connect to");
    prop_bool("ntp-sync", &ntp_sync_, "Synchronize time using NTP on the publisher side");
    prop_string("ntp-srvs", &ntp_srvs_, "NTP hosts and ports (comma separated host:port)");
    prop_string("pub-topic", &topic_, "The topic's name to publish");
    prop_uint("pub-wait-timeout", &pub_wait_s_, "Timeout (s) for the publish acknowledgement (QoS >= 1)");
    prop_bool("cleansession", &clean_, "When it is TRUE, the state information is discarded at connect and disconnect");
    prop_int("keep-alive-interval", &keepalive_, "The maximum time (s) between messages from this client");
    prop_uint("max-buffer-size", &max_buf_, "The maximum message payload size (0 = not fixed)");
    prop_int("num-buffers", &num_buffers_, "Number of (remaining) buffers to accept until sending EOS (-1 = unlimited)");
    prop_int("mqtt-qos", &qos_, "Quality of Service level (0: at most once, 1/2: at least once)");
    prop_readonly("published", [this] { return std::to_string(published_.load()); }, "nnsx: messages published");
  }

 protected:
  bool start() override {
    BaseSink::start();
    if (client_id_.empty()) client_id_ = default_client_id("sink");
    if (topic_.empty()) topic_ = client_id_ + "/topic";
    std::string err;
    client_ = std::make_unique<comm::MqttClient>();
    if (!client_->connect(host_, std::atoi(port_.c_str()), client_id_, keepalive_, clean_, 5000, &err)) {
      post_error("mqttsink: " + err);
      client_.reset();
      return false;
    }
    const int64_t off = ntp_sync_ ? ntp_offset_ns(ntp_srvs_) : 0;
    if (ntp_sync_ && off == 0) NNSX_LOGW(name(), "ntp-sync: no NTP server answered; using the local clock");
    base_epoch_ = epoch_ns() + off;
    ntp_off_ = off;
    remaining_ = num_buffers_;
    published_ = 0;
    return true;
  }
  bool stop() override {
    if (client_) client_->close();
    client_.reset();
    return true;
  }
  bool set_caps(const Caps& caps) override {
    caps_str_ = caps.to_string();
    if (caps_str_.size() >= kCapsLen) {
      post_error("mqttsink: caps string longer than the 512-byte header field");
      return false;
    }
    return true;
  }

  FlowReturn render(const BufferPtr& buf) override {
    if (remaining_ == 0) return FlowReturn::EOS;
    if (buf->mems.size() > kMaxMems) {
      post_error("mqttsink: more than 16 memories in a buffer");
      return FlowReturn::ERROR;
    }
    MqttHdr h;
    std::memset(&h, 0, sizeof(h));
    h.num_mems = static_cast<uint32_t>(buf->mems.size());
    size_t total = 0;
    for (size_t i = 0; i < buf->mems.size(); ++i) {
      h.size_mems[i] = buf->mems[i]->size();
      total += buf->mems[i]->size();
    }
    if (max_buf_ && total > max_buf_) {
      post_error(strfmt("mqttsink: payload ", total, " B exceeds max-buffer-size ", max_buf_));
      return FlowReturn::ERROR;
    }
    h.base_time_epoch = base_epoch_;
    h.sent_time_epoch = epoch_ns() + ntp_off_;
    h.duration = buf->duration < 0 ? kNone : static_cast<uint64_t>(buf->duration);
    h.dts = buf->dts < 0 ? kNone : static_cast<uint64_t>(buf->dts);
    h.pts = buf->pts < 0 ? kNone : static_cast<uint64_t>(buf->pts);
    std::memcpy(h.caps, caps_str_.data(), std::min(caps_str_.size(), kCapsLen - 1));
    body_.resize(total);
    size_t off = 0;
    for (auto& m : buf->mems) {
      if (m->size()) std::memcpy(&body_[off], m->map_host(), m->size());
      off += m->size();
    }
    if (!client_->publish2(topic_, &h, sizeof(h), body_.data(), body_.size(), qos_, false,
                           static_cast<int>(pub_wait_s_ * 1000))) {
      post_error("mqttsink: failed to publish to " + topic_);
      return FlowReturn::ERROR;
    }
    ++published_;
    if (debug_) NNSX_LOGI(name(), "published ", total, " B on ", topic_);
    if (remaining_ > 0 && --remaining_ == 0) return FlowReturn::EOS;
    return FlowReturn::OK;
  }

 private:
  bool debug_ = false, ntp_sync_ = false, clean_ = true;
  std::string client_id_, host_ = "127.0.0.1", port_ = "1883", ntp_srvs_ = "pool.ntp.org:123", topic_;
  unsigned pub_wait_s_ = 1, max_buf_ = 0;
  int keepalive_ = 60, num_buffers_ = -1, qos_ = 0;
  int64_t remaining_ = -1, base_epoch_ = 0, ntp_off_ = 0;
  std::string caps_str_, body_;
  std::unique_ptr<comm::MqttClient> client_;
  std::atomic<uint64_t> published_{0};
};

// =============================================================== mqttsrc ====
class MqttSrc : public BaseSrc {
 public:
  explicit MqttSrc(const std::string& name) : BaseSrc("mqttsrc", name, Caps::Any()) {
    prop_bool("debug", &debug_, "Produce extra verbose output for debug purpose");
    prop_string("client-id", &client_id_, "The client identifier passed to the server (broker)");
    prop_string("host", &host_, "Host (broker) to connect to");
    prop_string("port", &port_, "Network port of host (broker) to connect to");
    prop_string("sub-topic", &topic_, "The topic's name to subscribe (mandatory)");
    prop_int("sub-timeout", &sub_timeout_us_,
             "The timeout (in microseconds) for receiving a message from subscribed topic (the stream ends)");
    prop_bool("cleansession", &clean_, "When it is TRUE, the state information is discarded at connect and disconnect");
    prop_int("keep-alive-interval", &keepalive_, "The maximum time (s) between messages from this client");
    prop_int("mqtt-qos", &qos_, "Quality of Service level");
    prop_readonly("dumped", [this] { return std::to_string(dumped_.load()); },
                  "nnsx: messages dropped because they were sent before this source started");
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    if (topic_.empty()) {
      post_error("mqttsrc: sub-topic is mandatory");
      return false;
    }
    if (client_id_.empty()) client_id_ = default_client_id("src");
    std::string err;
    client_ = std::make_unique<comm::MqttClient>();
    if (!client_->connect(host_, std::atoi(port_.c_str()), client_id_, keepalive_, clean_, 5000, &err) ||
        !client_->subscribe(topic_, qos_)) {
      post_error("mqttsrc: " + (err.empty() ? "subscribe to " + topic_ + " failed" : err));
      client_.reset();
      return false;
    }
    base_epoch_ = epoch_ns();
    caps_str_.clear();
    have_pending_ = false;
    dumped_ = 0;
    return true;
  }
  void on_stop() override {
    if (client_) client_->close();
    client_.reset();
  }
  void on_unlock() override {
    if (client_) client_->close();
  }

  // the publisher's caps ride in every message header: wait for the first one
  bool negotiate() override {
    if (!have_pending_) {
      const FlowReturn r = next(&pending_);
      if (r != FlowReturn::OK) return false;
      have_pending_ = true;
    }
    return BaseSrc::negotiate();
  }
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_str_.empty() ? Caps::Any() : Caps::from_string(caps_str_);
    return filter ? c.intersect(*filter) : c;
  }

  FlowReturn create(BufferPtr* out) override {
    if (have_pending_) {
      have_pending_ = false;
      *out = pending_;
      pending_.reset();
      return FlowReturn::OK;
    }
    BufferPtr b;
    const FlowReturn r = next(&b);
    if (r == FlowReturn::OK) *out = b;
    return r;
  }

 private:
  // receive, validate and unpack one message (caps changes are pushed downstream)
  FlowReturn next(BufferPtr* out) {
    int64_t left_ms = std::max<int64_t>(sub_timeout_us_ / 1000, 1000);
    while (true) {
      comm::MqttMessage m;
      bool to = false;
      const int step = 100;
      if (!client_ || !client_->recv(&m, step, &to)) {
        if (flushing_.load()) return FlowReturn::FLUSHING;
        if (!to) {
          post_error("mqttsrc: connection to the broker lost");
          return FlowReturn::ERROR;
        }
        left_ms -= step;
        if (left_ms <= 0) {
          NNSX_LOGI(name(), "no message on ", topic_, " for ", sub_timeout_us_ / 1000, " ms: end of stream");
          return FlowReturn::EOS;
        }
        continue;
      }
      if (m.payload.size() < kHdrLen) continue;
      MqttHdr h;
      std::memcpy(&h, m.payload.data(), kHdrLen);
      if (h.num_mems > kMaxMems) continue;
      size_t total = 0;
      for (uint32_t i = 0; i < h.num_mems; ++i) total += h.size_mems[i];
      if (kHdrLen + total != m.payload.size()) continue;
      // a message sent before this source started comes from the past (retained): dump it
      if (h.sent_time_epoch < base_epoch_) {
        ++dumped_;
        continue;
      }
      const std::string caps(h.caps, strnlen(h.caps, kCapsLen));
      if (caps != caps_str_) {
        const bool first = caps_str_.empty();
        caps_str_ = caps;
        if (!first && negotiated_) src_pad()->push_event(Event::make_caps(Caps::from_string(caps_str_)));
      }
      auto whole = Memory::from_bytes(m.payload.data() + kHdrLen, total);
      auto b = make_buffer();
      size_t off = 0;
      for (uint32_t i = 0; i < h.num_mems; ++i) {
        b->mems.push_back(Memory::view(whole, off, h.size_mems[i]));
        off += h.size_mems[i];
      }
      // re-base the publisher's timestamps onto this pipeline's clock (mqttsrc.c:1380-1410)
      const int64_t diff = h.base_time_epoch - base_epoch_;
      if (h.pts != kNone && static_cast<int64_t>(h.pts) + diff >= 0) {
        b->pts = static_cast<int64_t>(h.pts) + diff;
        if (h.dts != kNone) b->dts = static_cast<int64_t>(h.dts) + diff;
      }
      if (h.duration != kNone) b->duration = static_cast<int64_t>(h.duration);
      if (debug_) NNSX_LOGI(name(), "received ", total, " B on ", m.topic);
      *out = b;
      return FlowReturn::OK;
    }
  }

  bool debug_ = false, clean_ = true;
  std::string client_id_, host_ = "127.0.0.1", port_ = "1883", topic_;
  int64_t sub_timeout_us_ = 10000000;
  int keepalive_ = 60, qos_ = 2;
  int64_t base_epoch_ = 0;
  std::string caps_str_;
  std::unique_ptr<comm::MqttClient> client_;
  BufferPtr pending_;
  bool have_pending_ = false;
  std::atomic<uint64_t> dumped_{0};
};

}  // namespace

void register_mqtt_elements() {
  register_element("mqttsink", "Sink/MQTT", "Publish incoming data streams as a MQTT topic",
                   [](const std::string& n) { return std::make_unique<MqttSink>(n); });
  register_element("mqttsrc", "Source/MQTT", "Subscribe a MQTT topic and push incoming data to the GStreamer pipeline",
                   [](const std::string& n) { return std::make_unique<MqttSrc>(n); });
}

}  // namespace nnsx
