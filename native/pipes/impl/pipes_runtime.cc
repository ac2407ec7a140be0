// hbmr Pipes child runtime (libhbmr_pipes): the C++ side of the Pipes task
// protocol that a CPU or GPU task binary links.
//
// Protocol semantics follow Hadoop Pipes (message codes of
// hadoop-1.0.3/src/mapred/org/apache/hadoop/mapred/pipes/BinaryProtocol.java:66-85;
// child runtime src/c++/pipes/impl/HadoopPipes.cc): the parent sends
// AUTHENTICATION_REQ, START, SET_JOB_CONF, then RUN_MAP (+ MAP_ITEMs when the
// parent reads the input) or RUN_REDUCE (+ REDUCE_KEY/REDUCE_VALUE), then
// CLOSE; the child answers with OUTPUT / PARTITIONED_OUTPUT / STATUS /
// PROGRESS / counters and DONE.  Framing: Hadoop VInts and VInt-prefixed
// strings (SerialUtils).  This is an independent implementation:
//   * HMAC-SHA1 + base64 are built in (no OpenSSL),
//   * the combiner buffer is keyed per partition so combined records keep
//     their partition,
//   * GPU binaries learn the device the scheduler chose from HBMR_GPU_DEVICE /
//     argv[1] (the fork always passed 0).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "hadoop/Pipes.hh"
#include "hadoop/SerialUtils.hh"
#include "hadoop/StringUtils.hh"
#include "hmac_sha1.h"

using HadoopUtils::deserializeFloat;
using HadoopUtils::deserializeInt;
using HadoopUtils::deserializeLong;
using HadoopUtils::deserializeString;
using HadoopUtils::serializeFloat;
using HadoopUtils::serializeInt;
using HadoopUtils::serializeLong;
using HadoopUtils::serializeString;
using std::string;
using std::vector;

namespace HadoopPipes {

enum Msg {
  START_MESSAGE = 0, SET_JOB_CONF = 1, SET_INPUT_TYPES = 2, RUN_MAP = 3, MAP_ITEM = 4,
  RUN_REDUCE = 5, REDUCE_KEY = 6, REDUCE_VALUE = 7, CLOSE = 8, ABORT = 9, AUTHENTICATION_REQ = 10,
  OUTPUT = 50, PARTITIONED_OUTPUT = 51, STATUS = 52, PROGRESS = 53, DONE = 54,
  REGISTER_COUNTER = 55, INCREMENT_COUNTER = 56, AUTHENTICATION_RESP = 57
};

static const int kProtocolVersion = 0;
static int g_argc = 0;
static char** g_argv = nullptr;

void setProgramArgs(int argc, char** argv) {
  g_argc = argc;
  g_argv = argv;
}

int getGPUDeviceId() {
  if (const char* e = getenv("HBMR_GPU_DEVICE")) return atoi(e);
  if (g_argc > 1 && g_argv != nullptr) return atoi(g_argv[1]);
  return -1;
}

bool isGPUTask() { return getGPUDeviceId() >= 0; }

// ---------------------------------------------------------------------------------------
class JobConfImpl : public JobConf {
 public:
  std::map<string, string> values;
  void set(const string& k, const string& v) { values[k] = v; }
  bool hasKey(const string& key) const override { return values.count(key) != 0; }
  const string& get(const string& key) const override {
    auto it = values.find(key);
    HADOOP_ASSERT(it != values.end(), "Key " + key + " not found in JobConf");
    return it->second;
  }
  int getInt(const string& key) const override { return HadoopUtils::toInt(get(key)); }
  float getFloat(const string& key) const override { return HadoopUtils::toFloat(get(key)); }
  bool getBoolean(const string& key) const override { return HadoopUtils::toBool(get(key)); }
};

// Upward (child → parent) messages.
class Uplink {
 public:
  explicit Uplink(HadoopUtils::OutStream* s) : out(s) {}
  void output(const string& k, const string& v) {
    serializeInt(OUTPUT, *out);
    serializeString(k, *out);
    serializeString(v, *out);
  }
  void partitionedOutput(int part, const string& k, const string& v) {
    serializeInt(PARTITIONED_OUTPUT, *out);
    serializeInt(part, *out);
    serializeString(k, *out);
    serializeString(v, *out);
  }
  void status(const string& msg) {
    serializeInt(STATUS, *out);
    serializeString(msg, *out);
    out->flush();
  }
  void progress(float p) {
    serializeInt(PROGRESS, *out);
    serializeFloat(p, *out);
    out->flush();
  }
  void done() {
    serializeInt(DONE, *out);
    out->flush();
  }
  void registerCounter(int id, const string& group, const string& name) {
    serializeInt(REGISTER_COUNTER, *out);
    serializeInt(id, *out);
    serializeString(group, *out);
    serializeString(name, *out);
  }
  void incrementCounter(int id, uint64_t amount) {
    serializeInt(INCREMENT_COUNTER, *out);
    serializeInt(id, *out);
    serializeLong((int64_t)amount, *out);
  }
  void authenticate(const string& digest) {
    serializeInt(AUTHENTICATION_RESP, *out);
    serializeString(digest, *out);
    out->flush();
  }
  void flush() { out->flush(); }

 private:
  HadoopUtils::OutStream* out;
};

// Sink for map output: straight up, or through the in-task combiner.
class OutputSink {
 public:
  virtual void emit(int part, const string& k, const string& v) = 0;
  virtual void flush() {}
  virtual ~OutputSink() {}
};

class DirectSink : public OutputSink {
 public:
  DirectSink(Uplink* up, bool partitioned) : up(up), partitioned(partitioned) {}
  void emit(int part, const string& k, const string& v) override {
    if (partitioned) up->partitionedOutput(part, k, v);
    else up->output(k, v);
  }

 private:
  Uplink* up;
  bool partitioned;
};

class TaskContextImpl;

// Buffers map output per (partition, key) up to a byte budget, then runs the
// job's combiner over each key's values and forwards the result.
class CombineSink : public OutputSink {
 public:
  CombineSink(TaskContextImpl* ctx, Reducer* combiner, OutputSink* next, size_t budget)
      : ctx(ctx), combiner(combiner), next(next), budget(budget) {}
  void emit(int part, const string& k, const string& v) override {
    auto& vals = buf[std::make_pair(part, k)];
    if (vals.empty()) bytes += k.size();
    vals.push_back(v);
    bytes += v.size();
    if (bytes >= budget) spill();
  }
  void flush() override { spill(); }
  void spill();

 private:
  TaskContextImpl* ctx;
  Reducer* combiner;
  OutputSink* next;
  size_t budget;
  size_t bytes = 0;
  std::map<std::pair<int, string>, vector<string>> buf;
};

class TaskContextImpl : public MapContext, public ReduceContext {
 public:
  TaskContextImpl(const Factory& f, HadoopUtils::InStream* in, Uplink* up)
      : factory(f), down(in), up(up) {}

  // ---- protocol ------------------------------------------------------------------------
  int readCommand() {
    const int cmd = deserializeInt(*down);
    if (!authDone && cmd != AUTHENTICATION_REQ) {
      std::cerr << "hbmr pipes: command " << cmd << " before authentication" << std::endl;
      exit(-1);
    }
    return cmd;
  }

  // Process control messages until a task (map/reduce) starts.
  void waitForTask() {
    while (!hasTask && !done) {
      const int cmd = readCommand();
      switch (cmd) {
        case AUTHENTICATION_REQ: {
          string digest, challenge;
          deserializeString(digest, *down);
          deserializeString(challenge, *down);
          authenticate(digest, challenge);
          break;
        }
        case START_MESSAGE: {
          const int v = deserializeInt(*down);
          HADOOP_ASSERT(v == kProtocolVersion, "unknown protocol version " + HadoopUtils::toString(v));
          break;
        }
        case SET_JOB_CONF: {
          // a reused child may get the next job's conf: start from scratch
          conf = JobConfImpl();
          const int n = deserializeInt(*down);
          for (int i = 0; i + 1 < n; i += 2) {
            string k, v;
            deserializeString(k, *down);
            deserializeString(v, *down);
            conf.set(k, v);
          }
          if (n % 2) {
            string dangling;
            deserializeString(dangling, *down);
          }
          break;
        }
        case SET_INPUT_TYPES:
          deserializeString(inputKeyClass, *down);
          deserializeString(inputValueClass, *down);
          break;
        case RUN_MAP: {
          deserializeString(inputSplit, *down);
          numReduces = deserializeInt(*down);
          pipedInput = deserializeInt(*down) != 0;
          setupMap();
          break;
        }
        case RUN_REDUCE: {
          reducePartition = deserializeInt(*down);
          pipedOutput = deserializeInt(*down) != 0;
          setupReduce();
          break;
        }
        case CLOSE:
          done = true;
          break;
        case ABORT:
          std::cerr << "hbmr pipes: aborted by parent" << std::endl;
          exit(-1);
        default:
          HADOOP_ASSERT(false, "unexpected command " + HadoopUtils::toString(cmd));
      }
    }
  }

  void authenticate(const string& digest, const string& challenge) {
    string password;
    if (const char* f = getenv("hadoop.pipes.shared.secret.location")) {
      std::ifstream in(f, std::ios::binary);
      password.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    }
    authDone = true;
    if (password.empty()) return;  // debug runs from a command file
    if (hbmr::createDigest(password, challenge) != digest) {
      std::cerr << "hbmr pipes: server failed to authenticate" << std::endl;
      exit(-1);
    }
    up->authenticate(hbmr::createDigest(password, digest));
  }

  void setupMap() {
    hasTask = true;
    isMap = true;
    if (!pipedInput) reader.reset(factory.createRecordReader(*this));
    mapper.reset(factory.createMapper(*this));
    direct.reset(new DirectSink(up, false));
    if (numReduces > 0) {
      partitioner.reset(factory.createPartitioner(*this));
      direct.reset(new DirectSink(up, partitioner != nullptr));
      combiner.reset(factory.createCombiner(*this));
      if (combiner) {
        size_t mb = conf.hasKey("io.sort.mb") ? (size_t)conf.getInt("io.sort.mb") : 100;
        sink.reset(new CombineSink(this, combiner.get(), direct.get(), mb << 20));
      }
    } else {
      writer.reset(factory.createRecordWriter(*(ReduceContext*)this));
    }
  }

  void setupReduce() {
    hasTask = true;
    isMap = false;
    reducer.reset(factory.createReducer(*this));
    if (!pipedOutput) writer.reset(factory.createRecordWriter(*this));
    direct.reset(new DirectSink(up, false));
  }

  // next map record; false at end of input
  bool nextMapRecord() {
    if (reader) {
      if (!reader->next(key, value)) return false;
      progressTick();
      return true;
    }
    while (true) {
      const int cmd = readCommand();
      if (cmd == MAP_ITEM) {
        deserializeString(key, *down);
        deserializeString(value, *down);
        return true;
      }
      if (cmd == CLOSE) return false;
      if (cmd == ABORT) exit(-1);
      HADOOP_ASSERT(false, "unexpected command in map " + HadoopUtils::toString(cmd));
    }
  }

  // next reduce key; false at CLOSE
  bool nextReduceKey() {
    if (pendingKey) {
      pendingKey = false;
      key.swap(nextKey);
      return true;
    }
    while (true) {
      const int cmd = readCommand();
      if (cmd == REDUCE_KEY) {
        deserializeString(key, *down);
        return true;
      }
      if (cmd == REDUCE_VALUE) {  // values of a key the reducer skipped
        deserializeString(value, *down);
        continue;
      }
      if (cmd == CLOSE) return false;
      if (cmd == ABORT) exit(-1);
      HADOOP_ASSERT(false, "unexpected command in reduce " + HadoopUtils::toString(cmd));
    }
  }

  bool nextValue() override {
    if (combining) return nextCombineValue();
    const int cmd = readCommand();
    if (cmd == REDUCE_VALUE) {
      deserializeString(value, *down);
      return true;
    }
    if (cmd == REDUCE_KEY) {
      // the current key stays visible to the reducer until it returns
      deserializeString(nextKey, *down);
      pendingKey = true;
      return false;
    }
    if (cmd == CLOSE) {
      closed = true;
      return false;
    }
    if (cmd == ABORT) exit(-1);
    HADOOP_ASSERT(false, "unexpected command in values " + HadoopUtils::toString(cmd));
    return false;
  }

  // Child reuse (hbmr.pipes.child.reuse, the Pipes analogue of
  // mapred.job.reuse.jvm.num.tasks): after DONE the child waits for the next
  // RUN_MAP / RUN_REDUCE (optionally after a new SET_JOB_CONF) on the same
  // connection instead of exiting, so a GPU binary keeps its HIP context and
  // device buffers across tasks; CLOSE ends it.
  void run() {
    while (true) {
      runOne();
      if (!hasTask || !conf.hasKey("hbmr.pipes.child.reuse") ||
          !conf.getBoolean("hbmr.pipes.child.reuse"))
        return;
      resetTask();
    }
  }

  void resetTask() {
    hasTask = false;
    closed = false;
    pendingKey = false;
    reader.reset();
    sink.reset();
    direct.reset();
    combiner.reset();
    partitioner.reset();
    writer.reset();
    mapper.reset();
    reducer.reset();
  }

  void runOne() {
    waitForTask();
    if (done && !hasTask) {
      up->done();
      return;
    }
    if (isMap) {
      while (nextMapRecord()) mapper->map(*this);
      mapper->close();
      if (sink) sink->flush();
      if (reader) reader->close();
      if (writer) writer->close();
      // piped input: the CLOSE was consumed by nextMapRecord
    } else {
      while (!closed && nextReduceKey()) {
        reducer->reduce(*this);
        // drain values the reducer did not consume
        while (!closed && !pendingKey && nextValue()) {
        }
      }
      reducer->close();
      if (writer) writer->close();
    }
    up->done();
  }

  // ---- TaskContext ------------------------------------------------------------------------
  const JobConf* getJobConf() override { return &conf; }
  const string& getInputKey() override { return key; }
  const string& getInputValue() override { return value; }
  const string& getInputSplit() override { return inputSplit; }
  const string& getInputKeyClass() override { return inputKeyClass; }
  const string& getInputValueClass() override { return inputValueClass; }

  void emit(const string& k, const string& v) override {
    if (combining) {
      combineOut->emit(combinePart, k, v);
      return;
    }
    if (isMap && numReduces == 0) {
      if (writer) writer->emit(k, v);
      else up->output(k, v);
      return;
    }
    if (!isMap) {
      if (writer) writer->emit(k, v);
      else up->output(k, v);
      return;
    }
    const int part = partitioner ? partitioner->partition(k, numReduces) : 0;
    if (sink) sink->emit(part, k, v);
    else direct->emit(part, k, v);
  }

  void progress() override { progressTick(); }

  void progressTick() {
    const uint64_t now = HadoopUtils::getCurrentMillis();
    if (now - lastProgress > 1000) {
      lastProgress = now;
      up->progress(reader ? reader->getProgress() : 0.0f);
    }
  }

  void setStatus(const string& status) override { up->status(status); }

  Counter* getCounter(const string& group, const string& name) override {
    const int id = (int)counters.size();
    counters.emplace_back(new Counter(id));
    up->registerCounter(id, group, name);
    return counters.back().get();
  }

  void incrementCounter(const Counter* counter, uint64_t amount) override {
    up->incrementCounter(counter->getId(), amount);
  }

  // combiner plumbing (CombineSink drives the combiner through this context)
  void runCombiner(Reducer* comb, int part, const string& k, vector<string>& vals,
                   OutputSink* out) {
    combining = true;
    combinePart = part;
    combineOut = out;
    combineVals = &vals;
    combineIdx = 0;
    const string savedKey = key, savedValue = value;
    key = k;
    comb->reduce(*this);
    key = savedKey;
    value = savedValue;
    combining = false;
  }

  bool nextCombineValue() {
    if (combineIdx >= combineVals->size()) return false;
    value = (*combineVals)[combineIdx++];
    return true;
  }

 private:
  const Factory& factory;
  HadoopUtils::InStream* down;
  Uplink* up;
  JobConfImpl conf;
  string key, nextKey, value, inputSplit, inputKeyClass, inputValueClass;
  int numReduces = 0, reducePartition = 0;
  bool pipedInput = true, pipedOutput = true;
  bool hasTask = false, isMap = true, done = false, closed = false, pendingKey = false;
  bool authDone = false;
  uint64_t lastProgress = 0;
  std::unique_ptr<RecordReader> reader;
  std::unique_ptr<Mapper> mapper;
  std::unique_ptr<Reducer> reducer, combiner;
  std::unique_ptr<Partitioner> partitioner;
  std::unique_ptr<RecordWriter> writer;
  std::unique_ptr<OutputSink> direct, sink;
  vector<std::unique_ptr<Counter>> counters;
  bool combining = false;
  int combinePart = 0;
  OutputSink* combineOut = nullptr;
  vector<string>* combineVals = nullptr;
  size_t combineIdx = 0;
};

void CombineSink::spill() {
  for (auto& kv : buf) ctx->runCombiner(combiner, kv.first.first, kv.first.second, kv.second, next);
  buf.clear();
  bytes = 0;
}

// ---- liveness: exit if the parent stops accepting connections (5 s × 3) ----------------
struct PingArgs {
  int port;
};

static void* pingThread(void* arg) {
  const int port = ((PingArgs*)arg)->port;
  int failures = 0;
  while (true) {
    sleep(5);
    const int s = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in addr;
    memset(&addr, 0, sizeof(addr));
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)port);
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (s < 0 || connect(s, (sockaddr*)&addr, sizeof(addr)) != 0) {
      if (++failures >= 3) {
        std::cerr << "hbmr pipes: parent unreachable, exiting" << std::endl;
        _exit(-1);
      }
    } else {
      failures = 0;
    }
    if (s >= 0) close(s);
  }
  return nullptr;
}

// ---------------------------------------------------------------------------
// Text protocol (HadoopPipes.cc TextProtocol / TextUpwardProtocol): with neither
// hadoop.pipes.command.port nor .file set, the child reads tab-separated text
// commands on stdin ("mapItem\tK\tV", "runMap\tSPLIT\tR\tPIPED", ...) and writes
// text replies on stdout ("output\tK\tV", "done", ...), for debugging a task
// binary by hand.  Instead of a second protocol implementation the text is
// translated to and from the binary stream by two bridge threads, so the task
// context runs exactly the code path it runs under the parent.
namespace {

string unescapeText(const string& s) {
  string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 1 < s.size()) {
      const char c = s[++i];
      o += c == 't' ? '\t' : c == 'n' ? '\n' : c;
    } else {
      o += s[i];
    }
  }
  return o;
}

string escapeText(const string& s) {
  string o;
  for (char c : s) {
    if (c == '\t') o += "\\t";
    else if (c == '\n') o += "\\n";
    else if (c == '\\') o += "\\\\";
    else o += c;
  }
  return o;
}

struct BridgeFds { int text_in; int bin_out; int bin_in; FILE* text_out; };

void* textDownThread(void* arg) {
  BridgeFds* b = (BridgeFds*)arg;
  FILE* in = fdopen(b->text_in, "r");
  FILE* outf = fdopen(b->bin_out, "wb");
  HadoopUtils::FileOutStream out;
  out.open(outf);
  serializeInt(AUTHENTICATION_REQ, out);   // no secret in text mode: auth is a no-op
  serializeString("", out);
  serializeString("", out);
  char* line = nullptr;
  size_t cap = 0;
  ssize_t n;
  while ((n = getline(&line, &cap, in)) > 0) {
    string l(line, (size_t)n);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    if (l.empty()) continue;
    std::vector<string> f(1);
    for (char ch : l) {   // keeps empty fields (an empty value is legal)
      if (ch == '\t') f.emplace_back();
      else f.back() += ch;
    }
    for (auto& x : f) x = unescapeText(x);
    const string& c = f[0];
    auto need = [&](size_t k) {
      HADOOP_ASSERT(f.size() >= k, "Short text protocol command " + c);
    };
    if (c == "start") { need(2); serializeInt(START_MESSAGE, out); serializeInt(HadoopUtils::toInt(f[1]), out); }
    else if (c == "setJobConf") {
      serializeInt(SET_JOB_CONF, out);
      serializeInt((int)f.size() - 1, out);
      for (size_t i = 1; i < f.size(); ++i) serializeString(f[i], out);
    } else if (c == "setInputTypes") { need(3); serializeInt(SET_INPUT_TYPES, out); serializeString(f[1], out); serializeString(f[2], out); }
    else if (c == "runMap") { need(4); serializeInt(RUN_MAP, out); serializeString(f[1], out); serializeInt(HadoopUtils::toInt(f[2]), out); serializeInt(HadoopUtils::toInt(f[3]), out); }
    else if (c == "mapItem") { need(3); serializeInt(MAP_ITEM, out); serializeString(f[1], out); serializeString(f[2], out); }
    else if (c == "runReduce") { need(3); serializeInt(RUN_REDUCE, out); serializeInt(HadoopUtils::toInt(f[1]), out); serializeInt(HadoopUtils::toInt(f[2]), out); }
    else if (c == "reduceKey") { need(2); serializeInt(REDUCE_KEY, out); serializeString(f[1], out); }
    else if (c == "reduceValue") { need(2); serializeInt(REDUCE_VALUE, out); serializeString(f[1], out); }
    else if (c == "close") { serializeInt(CLOSE, out); }
    else if (c == "abort") { serializeInt(ABORT, out); }
    else { std::cerr << "hbmr pipes: illegal text protocol command " << c << std::endl; }
    out.flush();
  }
  free(line);
  fclose(outf);
  fclose(in);
  return nullptr;
}

void* textUpThread(void* arg) {
  BridgeFds* b = (BridgeFds*)arg;
  FILE* inf = fdopen(b->bin_in, "rb");
  HadoopUtils::FileInStream in;
  in.open(inf);
  FILE* o = b->text_out;
  try {
    for (;;) {
      const int cmd = deserializeInt(in);
      string k, v;
      switch (cmd) {
        case OUTPUT:
          deserializeString(k, in); deserializeString(v, in);
          fprintf(o, "output\t%s\t%s\n", escapeText(k).c_str(), escapeText(v).c_str());
          break;
        case PARTITIONED_OUTPUT: {
          const int part = deserializeInt(in);
          deserializeString(k, in); deserializeString(v, in);
          fprintf(o, "partitionedOutput\t%d\t%s\t%s\n", part, escapeText(k).c_str(),
                  escapeText(v).c_str());
          break;
        }
        case STATUS: deserializeString(k, in); fprintf(o, "status\t%s\n", escapeText(k).c_str()); break;
        case PROGRESS: fprintf(o, "progress\t%f\n", deserializeFloat(in)); break;
        case DONE: fprintf(o, "done\n"); fflush(o); break;
        case REGISTER_COUNTER: {
          const int id = deserializeInt(in);
          deserializeString(k, in); deserializeString(v, in);
          fprintf(o, "registerCounter\t%d\t%s\t%s\n", id, escapeText(k).c_str(), escapeText(v).c_str());
          break;
        }
        case INCREMENT_COUNTER: {
          const int id = deserializeInt(in);
          fprintf(o, "incrementCounter\t%d\t%lld\n", id, (long long)deserializeLong(in));
          break;
        }
        case AUTHENTICATION_RESP: deserializeString(k, in); break;
        default: fprintf(o, "unknown\t%d\n", cmd); break;
      }
    }
  } catch (HadoopUtils::Error&) {
    // end of the binary stream: the task closed its output
  }
  fflush(o);
  fclose(inf);
  return nullptr;
}

}  // namespace

bool runTask(const Factory& factory) {
  pthread_t textThreads[2];
  bool textMode = false;
  try {
    FILE* in = nullptr;
    FILE* out = nullptr;
    int sock = -1;
    if (const char* portStr = getenv("hadoop.pipes.command.port")) {
      const int port = atoi(portStr);
      sock = socket(AF_INET, SOCK_STREAM, 0);
      HADOOP_ASSERT(sock >= 0, "socket() failed");
      sockaddr_in addr;
      memset(&addr, 0, sizeof(addr));
      addr.sin_family = AF_INET;
      addr.sin_port = htons((uint16_t)port);
      addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      HADOOP_ASSERT(connect(sock, (sockaddr*)&addr, sizeof(addr)) == 0,
                    "cannot connect to parent port " + string(portStr));
      int one = 1;
      setsockopt(sock, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      in = fdopen(sock, "rb");
      out = fdopen(dup(sock), "wb");
      setvbuf(in, nullptr, _IOFBF, 128 * 1024);
      setvbuf(out, nullptr, _IOFBF, 128 * 1024);
      static PingArgs args;
      args.port = port;
      pthread_t t;
      pthread_create(&t, nullptr, pingThread, &args);
      pthread_detach(t);
    } else if (const char* file = getenv("hadoop.pipes.command.file")) {
      in = fopen(file, "rb");
      const string outName = string(file) + ".out";
      out = fopen(outName.c_str(), "wb");
    } else {
      // text protocol on stdin/stdout through the bridge threads; a write to a
      // bridge pipe whose other end has closed (the task ended while a bridge
      // still had bytes in flight) must fail with EPIPE, not kill the process
      signal(SIGPIPE, SIG_IGN);
      int down[2], up[2];
      HADOOP_ASSERT(pipe(down) == 0 && pipe(up) == 0, "pipe() failed");
      static BridgeFds fds;
      fds = {dup(0), down[1], up[0], stdout};
      in = fdopen(down[0], "rb");
      out = fdopen(up[1], "wb");
      pthread_create(&textThreads[0], nullptr, textDownThread, &fds);
      pthread_create(&textThreads[1], nullptr, textUpThread, &fds);
      textMode = true;
    }
    HadoopUtils::FileInStream inStream;
    inStream.open(in);
    HadoopUtils::FileOutStream outStream;
    outStream.open(out);
    Uplink up(&outStream);
    {
      TaskContextImpl ctx(factory, &inStream, &up);
      ctx.run();
    }
    outStream.flush();
    fclose(in);
    fclose(out);
    if (textMode) {  // the up bridge drains and prints what is left; stdin may stay open
      pthread_join(textThreads[1], nullptr);
      pthread_detach(textThreads[0]);
    }
    return true;
  } catch (HadoopUtils::Error& e) {
    std::cerr << "hbmr pipes error: " << e.getMessage() << std::endl;
    return false;
  }
}

}  // namespace HadoopPipes
