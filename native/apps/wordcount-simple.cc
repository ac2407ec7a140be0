// Pipes WordCount (the job of hadoop-1.0.3/src/examples/pipes/impl/wordcount-simple.cc):
// map emits (word, "1") per whitespace-separated token, combiner/reducer sum.
#include <string>
#include <vector>

#include "hadoop/Pipes.hh"
#include "hadoop/StringUtils.hh"
#include "hadoop/TemplateFactory.hh"

class WordCountMap : public HadoopPipes::Mapper {
 public:
  HadoopPipes::TaskContext::Counter* inputWords;
  explicit WordCountMap(HadoopPipes::TaskContext& ctx) {
    inputWords = ctx.getCounter("WORDCOUNT", "INPUT_WORDS");
  }
  void map(HadoopPipes::MapContext& ctx) override {
    const std::string& line = ctx.getInputValue();
    size_t i = 0, n = line.size();
    while (i < n) {
      while (i < n && (line[i] == ' ' || line[i] == '\t')) ++i;
      size_t j = i;
      while (j < n && line[j] != ' ' && line[j] != '\t') ++j;
      if (j > i) {
        ctx.emit(line.substr(i, j - i), "1");
        ctx.incrementCounter(inputWords, 1);
      }
      i = j;
    }
  }
};

class WordCountReduce : public HadoopPipes::Reducer {
 public:
  HadoopPipes::TaskContext::Counter* outputWords;
  explicit WordCountReduce(HadoopPipes::TaskContext& ctx) {
    outputWords = ctx.getCounter("WORDCOUNT", "OUTPUT_WORDS");
  }
  void reduce(HadoopPipes::ReduceContext& ctx) override {
    int sum = 0;
    while (ctx.nextValue()) sum += HadoopUtils::toInt(ctx.getInputValue());
    ctx.emit(ctx.getInputKey(), HadoopUtils::toString(sum));
    ctx.incrementCounter(outputWords, 1);
  }
};

int main(int argc, char* argv[]) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<WordCountMap, WordCountReduce, void, WordCountReduce>())
             ? 0
             : 1;
}
