// Pipes WordCount that reads its split and writes its output in C++ (no Java
// record reader/writer; cf. src/examples/pipes/impl/wordcount-nopipe.cc).  The
// split arrives as a serialised FileSplit (Text path, long start, long length).
#include <stdio.h>
#include <sys/stat.h>

#include <string>

#include "hadoop/Pipes.hh"
#include "hadoop/SerialUtils.hh"
#include "hadoop/StringUtils.hh"
#include "hadoop/TemplateFactory.hh"

class Map : public HadoopPipes::Mapper {
 public:
  explicit Map(HadoopPipes::TaskContext&) {}
  void map(HadoopPipes::MapContext& ctx) override {
    for (const std::string& w : HadoopUtils::splitString(ctx.getInputValue(), " "))
      if (!w.empty()) ctx.emit(w, "1");
  }
};

class Reduce : public HadoopPipes::Reducer {
 public:
  explicit Reduce(HadoopPipes::TaskContext&) {}
  void reduce(HadoopPipes::ReduceContext& ctx) override {
    int sum = 0;
    while (ctx.nextValue()) sum += HadoopUtils::toInt(ctx.getInputValue());
    ctx.emit(ctx.getInputKey(), HadoopUtils::toString(sum));
  }
};

// Reads whole lines of [start, start+length) (a line straddling the end belongs here).
class LineReader : public HadoopPipes::RecordReader {
 public:
  explicit LineReader(HadoopPipes::MapContext& ctx) {
    HadoopUtils::StringInStream s(ctx.getInputSplit());
    std::string path;
    HadoopUtils::deserializeString(path, s);
    if (path.rfind("file:", 0) == 0) path = path.substr(5);
    unsigned char b[16];
    s.read(b, 16);
    start = end = 0;
    for (int i = 0; i < 8; ++i) start = (start << 8) | b[i];
    long len = 0;
    for (int i = 8; i < 16; ++i) len = (len << 8) | b[i];
    end = start + len;
    f = fopen(path.c_str(), "rb");
    HADOOP_ASSERT(f != NULL, "cannot open " + path);
    fseek(f, start, SEEK_SET);
    pos = start;
    if (start != 0) skipLine();
  }
  void skipLine() {
    int c;
    while ((c = fgetc(f)) != EOF) {
      ++pos;
      if (c == '\n') break;
    }
  }
  bool next(std::string& key, std::string& value) override {
    if (pos > end) return false;
    value.clear();
    int c;
    bool any = false;
    while ((c = fgetc(f)) != EOF) {
      any = true;
      ++pos;
      if (c == '\n') break;
      value.push_back((char)c);
    }
    if (!any) return false;
    key = HadoopUtils::toString((int)pos);
    return true;
  }
  float getProgress() override {
    return end > start ? (float)(pos - start) / (float)(end - start) : 1.0f;
  }
  void close() override {
    if (f) fclose(f);
    f = NULL;
  }
  ~LineReader() override { close(); }

 private:
  FILE* f;
  long start, end, pos;
};

class Writer : public HadoopPipes::RecordWriter {
 public:
  explicit Writer(HadoopPipes::ReduceContext& ctx) {
    const HadoopPipes::JobConf* conf = ctx.getJobConf();
    const std::string dir = conf->get("mapred.work.output.dir");
    mkdir(dir.c_str(), 0777);
    const std::string name = dir + "/part-" + conf->get("mapred.task.partition");
    f = fopen(name.c_str(), "wb");
    HADOOP_ASSERT(f != NULL, "cannot create " + name);
  }
  void emit(const std::string& key, const std::string& value) override {
    fprintf(f, "%s -> %s\n", key.c_str(), value.c_str());
  }
  void close() override {
    if (f) fclose(f);
    f = NULL;
  }
  ~Writer() override { close(); }

 private:
  FILE* f;
};

int main(int argc, char* argv[]) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<Map, Reduce, void, void, LineReader, Writer>())
             ? 0
             : 1;
}
