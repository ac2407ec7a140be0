// hbmr Pipes C++ API.
//
// Source-compatible with the Hadoop Pipes API a task binary is written
// against (hadoop-1.0.3/src/c++/pipes/api/hadoop/Pipes.hh: JobConf, TaskContext,
// MapContext, ReduceContext, Mapper, Reducer, Partitioner, RecordReader,
// RecordWriter, Factory, runTask) so existing Pipes programs build unchanged
// against libhbmr_pipes.a.  hbmr additions for GPU map tasks:
//   * getGPUDeviceId()  — the device the scheduler placed this attempt on
//     (argv[1] of a GPU binary, as the fork intended but never delivered:
//     PipesGPUMapRunner.java:64-79 always passed device 0);
//   * isGPUTask().
#ifndef HBMR_PIPES_HH
#define HBMR_PIPES_HH

#include <stdint.h>

#include <string>
#include <vector>

namespace HadoopPipes {

class JobConf {
 public:
  virtual bool hasKey(const std::string& key) const = 0;
  virtual const std::string& get(const std::string& key) const = 0;
  virtual int getInt(const std::string& key) const = 0;
  virtual float getFloat(const std::string& key) const = 0;
  virtual bool getBoolean(const std::string& key) const = 0;
  virtual ~JobConf() {}
};

class TaskContext {
 public:
  class Counter {
   public:
    explicit Counter(int counterId) : id(counterId) {}
    Counter(const Counter& c) : id(c.id) {}
    int getId() const { return id; }

   private:
    int id;
  };

  virtual const JobConf* getJobConf() = 0;
  virtual const std::string& getInputKey() = 0;
  virtual const std::string& getInputValue() = 0;
  virtual void emit(const std::string& key, const std::string& value) = 0;
  virtual void progress() = 0;
  virtual void setStatus(const std::string& status) = 0;
  virtual Counter* getCounter(const std::string& group, const std::string& name) = 0;
  virtual void incrementCounter(const Counter* counter, uint64_t amount) = 0;
  virtual ~TaskContext() {}
};

class MapContext : public TaskContext {
 public:
  virtual const std::string& getInputSplit() = 0;
  virtual const std::string& getInputKeyClass() = 0;
  virtual const std::string& getInputValueClass() = 0;
};

class ReduceContext : public TaskContext {
 public:
  virtual bool nextValue() = 0;
};

class Closable {
 public:
  virtual void close() {}
  virtual ~Closable() {}
};

class Mapper : public Closable {
 public:
  virtual void map(MapContext& context) = 0;
};

class Reducer : public Closable {
 public:
  virtual void reduce(ReduceContext& context) = 0;
};

class Partitioner {
 public:
  virtual int partition(const std::string& key, int numOfReduces) = 0;
  virtual ~Partitioner() {}
};

class RecordReader : public Closable {
 public:
  virtual bool next(std::string& key, std::string& value) = 0;
  virtual float getProgress() = 0;
};

class RecordWriter : public Closable {
 public:
  virtual void emit(const std::string& key, const std::string& value) = 0;
};

class Factory {
 public:
  virtual Mapper* createMapper(MapContext& context) const = 0;
  virtual Reducer* createReducer(ReduceContext& context) const = 0;
  virtual Reducer* createCombiner(MapContext& context) const { return NULL; }
  virtual Partitioner* createPartitioner(MapContext& context) const { return NULL; }
  virtual RecordReader* createRecordReader(MapContext& context) const { return NULL; }
  virtual RecordWriter* createRecordWriter(ReduceContext& context) const { return NULL; }
  virtual ~Factory() {}
};

// Run the task protocol loop until the parent says close; returns true on success.
bool runTask(const Factory& factory);

// hbmr: GPU placement of the current attempt (-1 for CPU attempts).
int getGPUDeviceId();
bool isGPUTask();
// hbmr: set by runTask from argv when a GPU binary is launched with a device id.
void setProgramArgs(int argc, char** argv);

}  // namespace HadoopPipes

#endif
