// oracle/oracle.cc — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT PATH.
//
// A faithful CPU restatement of OpenTSDB 1.1's query-time aggregation path,
// structured exactly like the reference's Java iterators so that every quirk
// is reproduced by construction. Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this (as the checker / CPU baseline);
// opentsdb_amd never does.
//
// Parity anchoring: the reference (Java, jars not vendored) cannot be built
// or run in this image. The restatement is pinned by the
// reference's own test vectors (TestAggregators.java:68-109,
// TestCompactionQueue.java:77-299) and by hand-derived known answers
// KA-1..KA-8 traced through the Java source, committed under
// tests/golden/.
//
// Java semantics restated: wrapping `long`, truncating `/`, `(long)double`
// saturating with NaN->0, strict IEEE double (compile with
// -ffp-contract=off), float->double widening, `short` iterator indices.
//
// File:line citations are relative to the reference root.

#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <queue>
#include <stdexcept>
#include <string>
#include <vector>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>

#include "../include/tsdbhip.h"

namespace oracle {

// ---------------------------------------------------------------- java ----
static inline int64_t ladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t lsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t lmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static inline int64_t ldiv(int64_t a, int64_t b) {  // Java: truncation, MIN/-1 = MIN
  if (b == -1) return (int64_t)(0 - (uint64_t)a);
  return a / b;
}
static inline int64_t d2l(double d) {  // Java (long) cast (JLS 5.1.3)
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
static inline int64_t dbits(double d) { int64_t b; std::memcpy(&b, &d, 8); return b; }
static inline double bitsd(int64_t b) { double d; std::memcpy(&d, &b, 8); return d; }

struct JavaException : std::runtime_error {
  int code;
  JavaException(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
static void illegal_data(const std::string& m) { throw JavaException(TSDBHIP_E_ILLEGAL_DATA, m); }
static void oob(const std::string& m) { throw JavaException(TSDBHIP_E_OUT_OF_BOUNDS, m); }

// org.hbase.async.Bytes big-endian getters (asynchbase 1.4.1; restated).
static inline void chk(const std::vector<uint8_t>& b, int64_t off, int n) {
  if (off < 0 || off + n > (int64_t)b.size()) oob("ArrayIndexOutOfBounds");
}
static inline int16_t getShort(const std::vector<uint8_t>& b, int64_t off) {
  chk(b, off, 2); return (int16_t)((b[off] << 8) | b[off + 1]);
}
static inline int32_t getUnsignedShort(const std::vector<uint8_t>& b, int64_t off) {
  chk(b, off, 2); return (b[off] << 8) | b[off + 1];
}
static inline int32_t getInt(const std::vector<uint8_t>& b, int64_t off) {
  chk(b, off, 4);
  return (int32_t)(((uint32_t)b[off] << 24) | ((uint32_t)b[off + 1] << 16) |
                   ((uint32_t)b[off + 2] << 8) | (uint32_t)b[off + 3]);
}
static inline int64_t getLong(const std::vector<uint8_t>& b, int64_t off) {
  chk(b, off, 8);
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v = (v << 8) | b[off + i];
  return (int64_t)v;
}
static inline void setShort(std::vector<uint8_t>& b, int16_t v, int64_t off) {
  b[off] = (uint8_t)((uint16_t)v >> 8); b[off + 1] = (uint8_t)v;
}

// Const.java:19-41
static const int FLAG_BITS = 4;
static const int FLAG_FLOAT = 0x8;
static const int LENGTH_MASK = 0x7;
static const int FLAGS_MASK = FLAG_FLOAT | LENGTH_MASK;

// A compacted HBase KeyValue as seen by Span.addRow: the only key field the
// path reads is base_time (Bytes.getUnsignedInt(key, metric_width)); span
// identity (metric+tags) is given by which span the row is handed to.
struct KeyValue {
  uint32_t base_time;
  std::vector<uint8_t> qualifier;
  std::vector<uint8_t> value;
  int32_t index = -1;  // position in the caller's row (compaction's keep/delete report)
};

// ------------------------------------------------------ DataPoint iface ---
struct DataPoint {
  virtual ~DataPoint() {}
  virtual int64_t timestamp() = 0;
  virtual bool isInteger() = 0;
  virtual int64_t longValue() = 0;
  virtual double doubleValue() = 0;
  virtual double toDouble() = 0;
};
struct SeekableView {
  virtual ~SeekableView() {}
  virtual bool hasNext() = 0;
  virtual DataPoint* next() = 0;
  virtual void seek(int64_t ts) = 0;
};
struct NoSuchElement : std::runtime_error { NoSuchElement() : std::runtime_error("no more elements") {} };

// Aggregator.java:24-86
struct Longs { virtual ~Longs() {} virtual bool hasNextValue() = 0; virtual int64_t nextLongValue() = 0; };
struct Doubles { virtual ~Doubles() {} virtual bool hasNextValue() = 0; virtual double nextDoubleValue() = 0; };

// Aggregators.java:76-243 (sum, min, max, avg, dev)
static int64_t runLong(int agg, Longs& v) {
  switch (agg) {
    case TSDBHIP_AGG_SUM: {  // :78-84
      int64_t r = v.nextLongValue();
      while (v.hasNextValue()) r = ladd(r, v.nextLongValue());
      return r;
    }
    case TSDBHIP_AGG_MIN: {  // :102-111
      int64_t m = v.nextLongValue();
      while (v.hasNextValue()) { int64_t x = v.nextLongValue(); if (x < m) m = x; }
      return m;
    }
    case TSDBHIP_AGG_MAX: {  // :132-141
      int64_t m = v.nextLongValue();
      while (v.hasNextValue()) { int64_t x = v.nextLongValue(); if (x > m) m = x; }
      return m;
    }
    case TSDBHIP_AGG_AVG: {  // :162-170  long sum / int n
      int64_t r = v.nextLongValue();
      int32_t n = 1;
      while (v.hasNextValue()) { r = ladd(r, v.nextLongValue()); n++; }
      return ldiv(r, (int64_t)n);
    }
    case TSDBHIP_AGG_DEV: {  // :198-217  Welford, population
      double old_mean = (double)v.nextLongValue();
      if (!v.hasNextValue()) return 0;
      int64_t n = 2;
      double new_mean = 0, variance = 0;
      do {
        const double x = (double)v.nextLongValue();
        new_mean = old_mean + (x - old_mean) / (double)n;
        variance += (x - old_mean) * (x - new_mean);
        old_mean = new_mean;
        n++;
      } while (v.hasNextValue());
      return d2l(std::sqrt(variance / (double)(n - 1)));
    }
  }
  throw JavaException(TSDBHIP_E_INVALID_ARG, "bad aggregator");
}
static double runDouble(int agg, Doubles& v) {
  switch (agg) {
    case TSDBHIP_AGG_SUM: {
      double r = v.nextDoubleValue();
      while (v.hasNextValue()) r += v.nextDoubleValue();
      return r;
    }
    case TSDBHIP_AGG_MIN: {
      double m = v.nextDoubleValue();
      while (v.hasNextValue()) { double x = v.nextDoubleValue(); if (x < m) m = x; }
      return m;
    }
    case TSDBHIP_AGG_MAX: {
      double m = v.nextDoubleValue();
      while (v.hasNextValue()) { double x = v.nextDoubleValue(); if (x > m) m = x; }
      return m;
    }
    case TSDBHIP_AGG_AVG: {
      double r = v.nextDoubleValue();
      int32_t n = 1;
      while (v.hasNextValue()) { r += v.nextDoubleValue(); n++; }
      return r / (double)n;
    }
    case TSDBHIP_AGG_DEV: {  // :219-238
      double old_mean = v.nextDoubleValue();
      if (!v.hasNextValue()) return 0;
      int64_t n = 2;
      double new_mean = 0, variance = 0;
      do {
        const double x = v.nextDoubleValue();
        new_mean = old_mean + (x - old_mean) / (double)n;
        variance += (x - old_mean) * (x - new_mean);
        old_mean = new_mean;
        n++;
      } while (v.hasNextValue());
      return std::sqrt(variance / (double)(n - 1));
    }
  }
  throw JavaException(TSDBHIP_E_INVALID_ARG, "bad aggregator");
}

// ---------------------------------------------------------------- RowSeq ---
// RowSeq.java:34-498
struct RowSeq {
  bool has_key = false;
  uint32_t base = 0;
  std::vector<uint8_t> qualifiers, values;

  void setRow(const KeyValue& row) {  // :70-78
    if (has_key) throw JavaException(TSDBHIP_E_INVALID_ARG, "setRow was already called");
    has_key = true; base = row.base_time; qualifiers = row.qualifier; values = row.value;
  }
  static bool canTimeDeltaFit(int64_t d) { return d < (1 << (16 - FLAG_BITS)); }  // :182-184
  int64_t baseTime() const { return base; }
  int size() const { return (int)(qualifiers.size() / 2); }
  int64_t timestamp(int i) const {  // :278-283
    if (i >= size() || i < 0) oob("index out of bounds");
    return baseTime() + (getUnsignedShort(qualifiers, i * 2) >> FLAG_BITS);
  }
  // :92-172
  void addRow(const KeyValue& row) {
    const int64_t base_time = row.base_time;
    const int32_t time_adj = (int32_t)(base_time - baseTime());
    if (time_adj <= 0) {
      // same key iff same span (identity given by the caller) and same base
      if (time_adj != 0) illegal_data("Attempt to add a row with a base_time <= baseTime()");
      has_key = false; qualifiers.clear(); values.clear();
      setRow(row);
      return;
    }
    const std::vector<uint8_t>& qual = row.qualifier;
    const int len = (int)qual.size();
    int last_delta = getUnsignedShort(qualifiers, (int64_t)qualifiers.size() - 2);
    last_delta >>= FLAG_BITS;
    const int old_qual_len = (int)qualifiers.size();
    std::vector<uint8_t> newquals(old_qual_len + len);
    std::memcpy(newquals.data(), qualifiers.data(), old_qual_len);
    for (int i = 0; i < len; i += 2) {
      int16_t qualifier = getShort(qual, i);
      const int time_delta = time_adj + ((qualifier & 0xFFFF) >> FLAG_BITS);
      if (!canTimeDeltaFit(time_delta)) illegal_data("time_delta too large");
      if (last_delta >= time_delta) return;  // LOG.error + ignore this row
      qualifier = (int16_t)((time_delta << FLAG_BITS) | (qualifier & FLAGS_MASK));
      setShort(newquals, qualifier, old_qual_len + i);
    }
    qualifiers.swap(newquals);
    const std::vector<uint8_t>& val = row.value;
    const int old_val_len = (int)values.size() - (old_qual_len == 2 ? 0 : 1);
    std::vector<uint8_t> newvals(old_val_len + val.size() + (len == 2 ? 1 : 0), 0);
    std::memcpy(newvals.data(), values.data(), old_val_len);
    std::memcpy(newvals.data() + old_val_len, val.data(), val.size());
    // assert newvals[last] == 0 (enabled in production, tsdb.in:86)
    if (newvals.empty() || newvals.back() != 0)
      throw JavaException(TSDBHIP_E_ILLEGAL_DATA, "AssertionError: Incorrect meta data byte after merge");
    values.swap(newvals);
  }

  // :194-206
  static int64_t extractIntegerValue(const std::vector<uint8_t>& values, int value_idx, int flags) {
    switch (flags & LENGTH_MASK) {
      case 7: return getLong(values, value_idx);
      case 3: return getInt(values, value_idx);
      case 1: return getShort(values, value_idx);
      case 0: chk(values, value_idx, 1); return (int8_t)values[value_idx];
    }
    illegal_data("Integer value not on 8/4/2/1 bytes");
    return 0;
  }
  // :216-226
  static double extractFloatingPointValue(const std::vector<uint8_t>& values, int value_idx, int flags) {
    switch (flags & LENGTH_MASK) {
      case 7: return bitsd(getLong(values, value_idx));
      case 3: { int32_t i = getInt(values, value_idx); float f; std::memcpy(&f, &i, 4); return (double)f; }
    }
    illegal_data("Floating point value not on 8 or 4 bytes");
    return 0;
  }

  // Iterator :360-497 — short qual_index/value_index, stale `qualifier`.
  struct Iterator : DataPoint {
    RowSeq* rs;
    int16_t qualifier = 0, qual_index = 0, value_index = 0;
    int64_t base_time;
    explicit Iterator(RowSeq* r) : rs(r), base_time(r->baseTime()) {}
    bool hasNext() const { return qual_index < (int)rs->qualifiers.size(); }
    DataPoint* next() {  // :385-395
      if (!hasNext()) throw NoSuchElement();
      qualifier = getShort(rs->qualifiers, qual_index);
      qual_index = (int16_t)(qual_index + 2);
      const int8_t flags = (int8_t)qualifier;
      value_index = (int16_t)(value_index + (flags & LENGTH_MASK) + 1);
      return this;
    }
    void seek(int64_t timestamp) {  // :405-421 incl. quirk Q1 (stale qualifier)
      if ((timestamp & (int64_t)0xFFFFFFFF00000000LL) != 0)
        throw JavaException(TSDBHIP_E_INVALID_ARG, "invalid timestamp");
      qual_index = 0;
      value_index = 0;
      const int len = (int)rs->qualifiers.size();
      while (qual_index < len && peekNextTimestamp() < timestamp) {
        qual_index = (int16_t)(qual_index + 2);
        const int8_t flags = (int8_t)qualifier;
        value_index = (int16_t)(value_index + (flags & LENGTH_MASK) + 1);
      }
      if (qual_index > 0) qualifier = getShort(rs->qualifiers, qual_index - 2);
    }
    int64_t timestamp() override { return base_time + ((qualifier & 0xFFFF) >> FLAG_BITS); }
    bool isInteger() override { return (qualifier & FLAG_FLOAT) == 0; }
    int64_t longValue() override {
      if (!isInteger()) throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
      const int8_t flags = (int8_t)qualifier;
      const int8_t vlen = (int8_t)((flags & LENGTH_MASK) + 1);
      return extractIntegerValue(rs->values, value_index - vlen, flags);
    }
    double doubleValue() override {
      if (isInteger()) throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
      const int8_t flags = (int8_t)qualifier;
      const int8_t vlen = (int8_t)((flags & LENGTH_MASK) + 1);
      return extractFloatingPointValue(rs->values, value_index - vlen, flags);
    }
    double toDouble() override { return isInteger() ? (double)longValue() : doubleValue(); }
    int32_t saveState() const { return ((int32_t)qual_index << 16) | (value_index & 0xFFFF); }
    void restoreState(int32_t state) {
      value_index = (int16_t)(state & 0xFFFF);
      state = (int32_t)((uint32_t)state >> 16);
      qual_index = (int16_t)state;
      qualifier = 0;
    }
    int64_t peekNextTimestamp() const {
      return base_time + (getUnsignedShort(rs->qualifiers, qual_index) >> FLAG_BITS);
    }
  };
};

// ------------------------------------------------------------------ Span ---
// Span.java:33-532
struct Span {
  std::vector<std::unique_ptr<RowSeq>> rows;

  int size() const { int s = 0; for (auto& r : rows) s += r->size(); return s; }
  // :87-132 (key mismatch checks omitted: span identity is given)
  void addRow(const KeyValue& row) {
    int64_t last_ts = 0;
    if (!rows.empty()) {
      RowSeq& last = *rows.back();
      last_ts = last.timestamp(last.size() - 1);
      if (RowSeq::canTimeDeltaFit(lastTimestampInRow(row) - last.baseTime())) {
        last.addRow(row);
        return;
      }
    }
    std::unique_ptr<RowSeq> rowseq(new RowSeq());
    rowseq->setRow(row);
    if (last_ts >= rowseq->timestamp(0)) return;  // LOG.error, dropped
    rows.push_back(std::move(rowseq));
  }
  static int64_t lastTimestampInRow(const KeyValue& row) {  // :141-148
    const int64_t base_time = row.base_time;
    const int16_t last_delta = (int16_t)(getUnsignedShort(row.qualifier, (int64_t)row.qualifier.size() - 2) >> FLAG_BITS);
    return base_time + last_delta;
  }
  int64_t timestamp(int i) const {  // :174-179 via getIdxOffsetFor
    int idx = 0, offset = 0;
    for (auto& r : rows) { int sz = r->size(); if (offset + sz > i) break; offset += sz; idx++; }
    if (idx >= (int)rows.size()) oob("index out of bounds");
    return rows[idx]->timestamp(i - offset);
  }
  int16_t seekRow(int64_t timestamp) const {  // :223-240
    int16_t row_index = 0;
    const int nrows = (int)rows.size();
    for (int i = 0; i < nrows; i++) {
      const RowSeq& row = *rows[i];
      const int sz = row.size();
      if (row.timestamp(sz - 1) < timestamp) row_index++;
      else break;
    }
    if (row_index == nrows) --row_index;
    return row_index;
  }

  // Iterator :248-294
  struct Iterator : SeekableView {
    Span* sp;
    int16_t row_index = 0;
    std::unique_ptr<RowSeq::Iterator> current_row;
    explicit Iterator(Span* s) : sp(s), current_row(new RowSeq::Iterator(s->rows[0].get())) {}
    bool hasNext() override {
      return current_row->hasNext() || row_index < (int)sp->rows.size() - 1;
    }
    DataPoint* next() override {
      if (current_row->hasNext()) return current_row->next();
      if (row_index < (int)sp->rows.size() - 1) {
        row_index++;
        current_row.reset(new RowSeq::Iterator(sp->rows[row_index].get()));
        return current_row->next();
      }
      throw NoSuchElement();
    }
    void seek(int64_t timestamp) override {
      int16_t ri = sp->seekRow(timestamp);
      if (ri != row_index) {
        row_index = ri;
        current_row.reset(new RowSeq::Iterator(sp->rows[ri].get()));
      }
      current_row->seek(timestamp);
    }
  };

  // DownsamplingIterator :309-530
  struct DownsamplingIterator : SeekableView, DataPoint, Longs, Doubles {
    static const int64_t FLAG_FLOAT_TS = (int64_t)0x8000000000000000ULL;
    static const int64_t TIME_MASK = 0x7FFFFFFFFFFFFFFFLL;
    Span* sp;
    int interval;
    int ds;
    int16_t row_index = 0;
    std::unique_ptr<RowSeq::Iterator> current_row;
    int64_t time = 0;
    int64_t value = 0;
    DownsamplingIterator(Span* s, int iv, int agg)
        : sp(s), interval(iv), ds(agg), current_row(new RowSeq::Iterator(s->rows[0].get())) {}

    bool hasNext() override {
      return current_row->hasNext() || row_index < (int)sp->rows.size() - 1;
    }
    bool moveToNext() {  // :362-375
      if (!current_row->hasNext()) {
        if (row_index < (int)sp->rows.size() - 1) {
          current_row.reset(new RowSeq::Iterator(sp->rows[++row_index].get()));
          current_row->next();
          return true;
        }
        return false;
      }
      current_row->next();
      return true;
    }
    DataPoint* next() override {  // :377-422
      if (!hasNext()) throw NoSuchElement();
      int64_t newtime = 0;
      const int16_t saved_row_index = row_index;
      const int32_t saved_state = current_row->saveState();
      moveToNext();
      time = current_row->timestamp() + interval;
      bool integer = true;
      int32_t npoints = 0;
      do {
        npoints++;
        newtime += current_row->timestamp();
        integer &= current_row->isInteger();
      } while (moveToNext() && current_row->timestamp() < time);
      newtime /= npoints;
      if (row_index != saved_row_index) {
        row_index = saved_row_index;
        current_row.reset(new RowSeq::Iterator(sp->rows[row_index].get()));
      }
      current_row->restoreState(saved_state);
      if (integer) value = runLong(ds, *(Longs*)this);
      else value = dbits(runDouble(ds, *(Doubles*)this));
      time = newtime;
      if (!integer) time |= FLAG_FLOAT_TS;
      return this;
    }
    void seek(int64_t timestamp) override {  // :432-440
      int16_t ri = sp->seekRow(timestamp);
      if (ri != row_index) {
        row_index = ri;
        current_row.reset(new RowSeq::Iterator(sp->rows[ri].get()));
      }
      current_row->seek(timestamp);
    }
    int64_t timestamp() override { return time & TIME_MASK; }
    bool isInteger() override { return (time & FLAG_FLOAT_TS) == 0; }
    int64_t longValue() override {
      if (isInteger()) return value;
      throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
    }
    double doubleValue() override {
      if (!isInteger()) return bitsd(value);
      throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
    }
    double toDouble() override { return isInteger() ? (double)longValue() : doubleValue(); }
    bool hasNextValue() override {  // :476-488
      if (!current_row->hasNext()) {
        if (row_index < (int)sp->rows.size() - 1)
          return sp->rows[row_index + 1]->timestamp(0) < time;
        return false;
      }
      return current_row->peekNextTimestamp() < time;
    }
    int64_t nextLongValue() override {
      if (hasNextValue()) { moveToNext(); return current_row->longValue(); }
      throw NoSuchElement();
    }
    double nextDoubleValue() override {
      if (hasNextValue()) { moveToNext(); return current_row->toDouble(); }
      throw NoSuchElement();
    }
  };
};

// ------------------------------------------------------------- SpanGroup ---
// SpanGroup.java:46-816
struct SpanGroup {
  int64_t start_time, end_time;
  std::vector<Span*> spans;
  bool rate;
  int aggregator;
  int downsampler;
  int sample_interval;

  void add(Span* span) {  // :130-142
    if (span->timestamp(0) <= end_time && span->timestamp(span->size() - 1) >= start_time)
      spans.push_back(span);
  }
  int aggregatedSize() const { int s = 0; for (auto* sp : spans) s += sp->size(); return s; }

  struct SGIterator : DataPoint, Longs, Doubles {
    static const int64_t FLAG_FLOAT_TS = (int64_t)0x8000000000000000ULL;
    static const int64_t TIME_MASK = 0x7FFFFFFFFFFFFFFFLL;
    SpanGroup* g;
    std::vector<std::unique_ptr<SeekableView>> iterators;
    std::vector<int64_t> timestamps, values;
    int current = 0;
    int pos = 0;

    explicit SGIterator(SpanGroup* grp) : g(grp) {  // :435-475
      const int size = (int)g->spans.size();
      iterators.resize(size);
      timestamps.assign(size * (g->rate ? 3 : 2), 0);
      values.assign(size * (g->rate ? 3 : 2), 0);
      for (int i = 0; i < size; i++) {
        SeekableView* it;
        if (g->downsampler < 0) it = new Span::Iterator(g->spans[i]);
        else it = new Span::DownsamplingIterator(g->spans[i], g->sample_interval, g->downsampler);
        iterators[i].reset(it);
        it->seek(g->start_time);
        DataPoint* dp;
        try {
          dp = it->next();
        } catch (NoSuchElement&) {
          throw JavaException(TSDBHIP_E_EMPTY_SPAN, "AssertionError: Span is empty!");
        }
        if (dp->timestamp() >= g->start_time) {
          putDataPoint(size + i, dp);
        } else {
          endReached(i);
          continue;
        }
        if (g->rate) {
          if (it->hasNext()) moveToNext(i);
          else endReached(i);
        }
      }
    }
    void endReached(int i) {
      timestamps[iterators.size() + i] = TIME_MASK;
      iterators[i].reset();
    }
    void putDataPoint(int i, DataPoint* dp) {  // :492-504
      timestamps[i] = dp->timestamp();
      if (dp->isInteger()) {
        values[i] = dp->longValue();
      } else {
        values[i] = dbits(dp->doubleValue());
        timestamps[i] |= FLAG_FLOAT_TS;
      }
    }
    bool hasNext() {  // :510-522
      const int size = (int)iterators.size();
      for (int i = 0; i < size; i++)
        if ((timestamps[size + i] & TIME_MASK) <= g->end_time) return true;
      return false;
    }
    void next() {  // :524-577
      const int size = (int)iterators.size();
      int64_t min_ts = INT64_MAX;
      for (int i = current; i < size; i++)
        if (timestamps[i + size] == TIME_MASK) timestamps[i] = 0;
      current = -1;
      bool multiple = false;
      for (int i = 0; i < size; i++) {
        const int64_t ts = timestamps[size + i] & TIME_MASK;
        if (ts <= g->end_time) {
          if (ts < min_ts) { min_ts = ts; current = i; multiple = false; }
          else if (ts == min_ts) multiple = true;
        }
      }
      if (current < 0) throw NoSuchElement();
      moveToNext(current);
      if (multiple) {
        for (int i = current + 1; i < size; i++) {
          const int64_t ts = timestamps[size + i] & TIME_MASK;
          if (ts == min_ts) moveToNext(i);
        }
      }
    }
    void moveToNext(int i) {  // :583-608
      const int size = (int)iterators.size();
      const int nxt = size + i;
      if (g->rate) {
        timestamps[nxt + size] = timestamps[i];
        values[nxt + size] = values[i];
      }
      timestamps[i] = timestamps[nxt];
      values[i] = values[nxt];
      SeekableView* it = iterators[i].get();
      if (it->hasNext()) putDataPoint(nxt, it->next());
      else endReached(i);
    }
    int64_t timestamp() override { return timestamps[current] & TIME_MASK; }
    bool isInteger() override {  // :632-645
      if (g->rate) return false;
      for (int i = (int)timestamps.size() - 1; i >= 0; i--)
        if ((timestamps[i] & FLAG_FLOAT_TS) == FLAG_FLOAT_TS) return false;
      return true;
    }
    int64_t longValue() override {  // :647-653
      if (isInteger()) { pos = -1; return runLong(g->aggregator, *(Longs*)this); }
      throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
    }
    double doubleValue() override {  // :655-667
      if (!isInteger()) {
        pos = -1;
        const double value = runDouble(g->aggregator, *(Doubles*)this);
        if (value != value || std::isinf(value))
          throw JavaException(TSDBHIP_E_NAN_INF, "Got NaN or Infinity");
        return value;
      }
      throw JavaException(TSDBHIP_E_INVALID_ARG, "ClassCastException");
    }
    double toDouble() override { throw JavaException(TSDBHIP_E_INVALID_ARG, "Q4: inverted toDouble"); }
    bool hasNextValue(bool update_pos) {  // :687-700
      const int size = (int)iterators.size();
      for (int i = pos + 1; i < size; i++) {
        if (timestamps[i] != 0) { if (update_pos) pos = i; return true; }
      }
      return false;
    }
    bool hasNextValue() override { return hasNextValue(false); }
    int64_t nextLongValue() override {  // :702-730 (S12)
      if (hasNextValue(true)) {
        const int64_t y0 = values[pos];
        if (g->rate) throw JavaException(TSDBHIP_E_INVALID_ARG, "AssertionError: impossible");
        if (current == pos) return y0;
        const int64_t x = timestamps[current] & TIME_MASK;
        const int64_t x0 = timestamps[pos] & TIME_MASK;
        if (x == x0) return y0;
        const int size = (int)iterators.size();
        const int64_t y1 = values[pos + size];
        const int64_t x1 = timestamps[pos + size] & TIME_MASK;
        if (x == x1) return y1;
        const int64_t r = ladd(y0, ldiv(lmul(lsub(x, x0), lsub(y1, y0)), lsub(x1, x0)));
        if ((x1 & (int64_t)0xFFFFFFFF00000000LL) != 0)
          throw JavaException(TSDBHIP_E_INVALID_ARG, "AssertionError: x1 out of range");
        return r;
      }
      throw NoSuchElement();
    }
    double nextDoubleValue() override {  // :736-784 (S13)
      if (hasNextValue(true)) {
        const double y0 = ((timestamps[pos] & FLAG_FLOAT_TS) == FLAG_FLOAT_TS)
                              ? bitsd(values[pos]) : (double)values[pos];
        const int size = (int)iterators.size();
        if (g->rate) {
          const int64_t x0 = timestamps[pos] & TIME_MASK;
          const int prev = pos + size * 2;
          const double y1 = ((timestamps[prev] & FLAG_FLOAT_TS) == FLAG_FLOAT_TS)
                                ? bitsd(values[prev]) : (double)values[prev];
          const int64_t x1 = timestamps[prev] & TIME_MASK;
          if (!(x0 > x1)) throw JavaException(TSDBHIP_E_INVALID_ARG, "AssertionError: x0 > x1");
          return (y0 - y1) / (double)(x0 - x1);
        }
        if (current == pos) return y0;
        const int64_t x = timestamps[current] & TIME_MASK;
        const int64_t x0 = timestamps[pos] & TIME_MASK;
        if (x == x0) return y0;
        const int nxt = pos + size;
        const double y1 = ((timestamps[nxt] & FLAG_FLOAT_TS) == FLAG_FLOAT_TS)
                              ? bitsd(values[nxt]) : (double)values[nxt];
        const int64_t x1 = timestamps[nxt] & TIME_MASK;
        if (x == x1) return y1;
        const double r = y0 + ((double)(x - x0) * (y1 - y0)) / (double)(x1 - x0);
        if ((x1 & (int64_t)0xFFFFFFFF00000000LL) != 0)
          throw JavaException(TSDBHIP_E_INVALID_ARG, "AssertionError: x1 out of range");
        return r;
      }
      throw NoSuchElement();
    }
  };
};

// ----------------------------------------------------- CompactionQueue ---
// CompactionQueue.java:243-743 — the value of compacted[0] for one row.
struct CompactResult {
  int status = TSDBHIP_ROW_NONE;
  std::vector<uint8_t> qual, val;
  bool write = false;  // tsdb.put of the compacted cell (:276, :388-396, :422-427)
  int32_t keep = -1;   // KeyValue.index of the dup the row must not delete (:399)
};

static uint8_t fixQualifierFlags(uint8_t flags, int val_len) {  // :490-499
  return (uint8_t)((flags & ~(FLAGS_MASK >> 1)) | (val_len - 1));
}
static bool floatingPointValueToFix(uint8_t flags, const std::vector<uint8_t>& value) {  // :510-515
  return (flags & FLAG_FLOAT) != 0 && (flags & LENGTH_MASK) == 0x3 && value.size() == 8;
}
static std::vector<uint8_t> fixFloatingPointValue(uint8_t flags, const std::vector<uint8_t>& value) {  // :530-544
  if (floatingPointValueToFix(flags, value)) {
    if (value[0] == 0 && value[1] == 0 && value[2] == 0 && value[3] == 0)
      return std::vector<uint8_t>(value.begin() + 4, value.end());
    illegal_data("Corrupted floating point value");
  }
  return value;
}
struct Cell { std::vector<uint8_t> q, v; bool skip = false; };
static int memcmp_u(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {  // Bytes.memcmp
  const size_t n = std::min(a.size(), b.size());
  for (size_t i = 0; i < n; i++) if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  return (int)a.size() - (int)b.size();
}
static std::vector<Cell> breakDownValues(const std::vector<KeyValue>& row) {  // :690-743
  std::vector<Cell> cells;
  for (const KeyValue& kv : row) {
    const std::vector<uint8_t>& qual = kv.qualifier;
    const int len = (int)qual.size();
    const std::vector<uint8_t>& val = kv.value;
    if (len == 2) {
      std::vector<uint8_t> actual_val = fixFloatingPointValue(qual[1], val);
      const uint8_t q = fixQualifierFlags(qual[1], (int)actual_val.size());
      Cell c; c.q = {qual[0], q}; c.v = actual_val;
      cells.push_back(c);
      continue;
    }
    if (val.empty()) oob("ArrayIndexOutOfBounds");
    if (val[val.size() - 1] != 0) illegal_data("Don't know how to read this value");
    size_t val_idx = 0;
    for (int i = 0; i < len; i += 2) {
      Cell c; c.q = {qual[i], qual[i + 1]};
      const int vlen = (qual[i + 1] & LENGTH_MASK) + 1;
      if (val_idx + vlen > val.size()) oob("ArrayIndexOutOfBounds");
      c.v.assign(val.begin() + val_idx, val.begin() + val_idx + vlen);
      val_idx += vlen;
      cells.push_back(c);
    }
    if (val_idx != val.size() - 1) illegal_data("Corrupted value: couldn't break down");
  }
  return cells;
}
static thread_local bool g_entered_complex = false;  // rows that reached complexCompact
static CompactResult complexCompact(const std::vector<KeyValue>& row) {  // :600-679
  g_entered_complex = true;
  std::vector<Cell> cells = breakDownValues(row);
  std::stable_sort(cells.begin(), cells.end(),
                   [](const Cell& a, const Cell& b) { return memcmp_u(a.q, b.q) < 0; });
  int val_len = 1;
  int last_delta = -1;
  const int ncells = (int)cells.size();
  for (int i = 0; i < ncells; i++) {
    Cell& cell = cells[i];
    const int delta = (int16_t)((((cell.q[0] << 8) | cell.q[1]) & 0xFFFF) >> FLAG_BITS);
    if (delta == last_delta) {
      int j = i - 1;
      while (cells[j].skip) j--;
      const Cell& prev = cells[j];
      if (cell.q[1] != prev.q[1] || cell.v != prev.v) illegal_data("Found out of order or duplicate data");
      cell.skip = true;
      continue;
    }
    last_delta = delta;
    val_len += (int)cell.v.size();
  }
  CompactResult r;
  r.status = TSDBHIP_ROW_COMPLEX;
  for (const Cell& c : cells) {
    if (c.skip) continue;
    r.qual.insert(r.qual.end(), c.q.begin(), c.q.end());
    r.val.insert(r.val.end(), c.v.begin(), c.v.end());
  }
  r.val.push_back(0);
  (void)val_len;
  return r;
}
static CompactResult compact(std::vector<KeyValue> row) {  // :243-405 (compacted != null)
  CompactResult r;
  if (row.size() <= 1) {
    if (row.empty()) return r;
    KeyValue kv = row[0];
    const std::vector<uint8_t>& qual = kv.qualifier;
    if (qual.size() % 2 != 0 || qual.empty()) return r;
    const std::vector<uint8_t>& val = kv.value;
    if (qual.size() == 2 && floatingPointValueToFix(qual[1], val)) {
      std::vector<uint8_t> newval = fixFloatingPointValue(qual[1], val);
      r.qual = {qual[0], fixQualifierFlags(qual[1], (int)newval.size())};
      r.val = newval;
    } else {
      r.qual = qual; r.val = val;
    }
    r.status = TSDBHIP_ROW_SINGLE;
    return r;
  }
  bool trivial = true;
  int qual_len = 0, val_len = 1;
  int last_delta = -1;
  KeyValue longest = row[0];  // :283-284 (taken before any junk is dropped)
  size_t longest_len = longest.qualifier.size();
  int nkvs = (int)row.size();
  for (int i = 0; i < nkvs; i++) {
    const KeyValue& kv = row[i];
    const std::vector<uint8_t>& qual = kv.qualifier;
    const int len = (int)qual.size();
    if (len != 2) {
      if (len % 2 != 0 || len == 0) {
        row.erase(row.begin() + i); nkvs--; i--; continue;
      }
      trivial = false;
      if ((size_t)len > longest_len) {  // :309-312
        longest = kv;
        longest_len = (size_t)len;
      }
    } else {
      const int delta = (int16_t)((((qual[0] << 8) | qual[1]) & 0xFFFF) >> FLAG_BITS);
      if (delta <= last_delta) illegal_data("Found out of order or duplicate data");
      last_delta = delta;
      val_len += floatingPointValueToFix(qual[1], kv.value) ? 4 : (int)kv.value.size();
    }
    qual_len += len;
  }
  if (row.size() < 2) {
    if (row.empty()) return r;
    return compact(row);
  }
  if (trivial) {  // trivialCompact :450-474
    r.status = TSDBHIP_ROW_TRIVIAL;
    for (const KeyValue& kv : row) {
      std::vector<uint8_t> v = fixFloatingPointValue(kv.qualifier[1], kv.value);
      r.qual.push_back(kv.qualifier[0]);
      r.qual.push_back(fixQualifierFlags(kv.qualifier[1], (int)v.size()));
      r.val.insert(r.val.end(), v.begin(), v.end());
    }
    r.val.push_back(0);
    r.write = true;  // :276, never a dup: the compacted qualifier is longer than every KV's
    return r;
  }
  r = complexCompact(row);
  r.write = true;
  // :364-400 — does a KV of the row already hold the compacted qualifier?
  // `longest` is row[0] of the list before junk removal, replaced by each
  // later non-2-byte KV with a strictly longer qualifier (:283-312).
  if (r.qual.size() <= longest_len) {
    const KeyValue* dup = nullptr;
    if (longest.qualifier == r.qual) {
      dup = &longest;
    } else {
      for (const KeyValue& kv : row)  // (junk already removed, :302)
        if (kv.qualifier == r.qual) { dup = &kv; break; }
    }
    if (dup) {
      if (dup->value == r.val) r.write = false;  // :391-396
      r.keep = dup->index;                        // :399 row.remove(dup_idx)
    }
  }
  return r;
}

}  // namespace oracle

// ======================================================== C entry points ===
using namespace oracle;

static std::vector<uint8_t> slice(const uint8_t* base, uint64_t off, uint64_t n) {
  return std::vector<uint8_t>(base + off, base + off + n);
}

extern "C" {

int oracle_abi_version(void) { return TSDBHIP_ABI_VERSION; }

// Seconds spent in the last oracle_spangroup_run of this thread, split into
// Span assembly (Span.addRow over the KeyValues) and SpanGroup iteration.
static thread_local double t_assemble = 0, t_iterate = 0;
void oracle_last_seconds(double* assemble, double* iterate) { *assemble = t_assemble; *iterate = t_iterate; }

// Runs one SpanGroup exactly as GraphHandler.respondAsciiQuery consumes it
// (GraphHandler.java:791-808): for each point timestamp(), isInteger(),
// then longValue() or doubleValue(). Host pointers only.
int oracle_spangroup_run(const tsdbhip_sg_desc* d, tsdbhip_sg_out* out) {
  out->n_out = 0;
  out->n_input_points = 0;
  out->err_code = 0;
  out->err_index = -1;
  int64_t emitted = 0;
  auto t0 = std::chrono::steady_clock::now();
  auto t1 = t0;
  t_assemble = t_iterate = 0;
  try {
    // TsdbQuery.findSpans (TsdbQuery.java:240-285) hands the scanner's rows to
    // Span.addRow in row-key order: metric | base_time | tags, i.e. by base
    // time, then span (TreeMap order of the tags). A merge of the spans' row
    // sequences (each span's own rows in the order given).
    std::vector<std::unique_ptr<Span>> spans(d->n_spans);
    std::vector<uint64_t> next(d->n_spans);
    using Head = std::pair<std::pair<uint32_t, uint32_t>, uint64_t>;  // ((base, span), row)
    std::priority_queue<Head, std::vector<Head>, std::greater<Head>> heads;
    for (uint32_t s = 0; s < d->n_spans; s++) {
      spans[s].reset(new Span());
      next[s] = d->span_row_start[s];
      if (next[s] < d->span_row_start[s + 1]) heads.push({{d->row_base[next[s]], s}, next[s]});
    }
    while (!heads.empty()) {
      const Head e = heads.top();
      heads.pop();
      const uint64_t r = e.second;
      const uint32_t s = e.first.second;
      KeyValue kv;
      kv.base_time = d->row_base[r];
      kv.qualifier = slice(d->qual_bytes, d->row_qual_off[r], (uint64_t)d->row_ncells[r] * 2);
      kv.value = slice(d->val_bytes, d->row_val_off[r], d->row_val_len[r]);
      if (++next[s] < d->span_row_start[s + 1]) heads.push({{d->row_base[next[s]], s}, next[s]});
      spans[s]->addRow(kv);
    }
    SpanGroup g;
    g.start_time = d->start_time;
    g.end_time = d->end_time;
    g.rate = d->rate != 0;
    g.aggregator = d->agg;
    g.downsampler = d->ds_interval > 0 ? d->ds_agg : -1;
    g.sample_interval = d->ds_interval;
    for (auto& sp : spans) {
      if (sp->rows.empty() || sp->size() == 0)
        throw JavaException(TSDBHIP_E_EMPTY_SPAN, "IndexOutOfBounds: empty span");
      g.add(sp.get());
    }
    out->n_input_points = (uint64_t)g.aggregatedSize();
    t1 = std::chrono::steady_clock::now();
    t_assemble = std::chrono::duration<double>(t1 - t0).count();
    SpanGroup::SGIterator it(&g);
    while (it.hasNext()) {
      it.next();
      const int64_t ts = it.timestamp();
      const bool isint = it.isInteger();
      const int64_t bits = isint ? it.longValue() : dbits(it.doubleValue());
      if ((uint64_t)emitted >= out->capacity) {
        out->err_code = TSDBHIP_E_CAPACITY;
        return TSDBHIP_E_CAPACITY;
      }
      out->ts[emitted] = ts;
      out->is_int[emitted] = isint ? 1 : 0;
      out->bits[emitted] = bits;
      emitted++;
      out->n_out = (uint64_t)emitted;
    }
    t_iterate = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
  } catch (JavaException& e) {
    out->err_code = e.code;
    out->err_index = emitted;
    return e.code;
  } catch (NoSuchElement&) {
    out->err_code = TSDBHIP_E_INVALID_ARG;
    out->err_index = emitted;
    return TSDBHIP_E_INVALID_ARG;
  }
  return TSDBHIP_OK;
}

// Aggregators over a plain sequence (TestAggregators' Numbers fake,
// TestAggregators.java:39-65).
struct SeqLongs : Longs {
  const int64_t* v; size_t n, i = 0;
  SeqLongs(const int64_t* a, size_t b) : v(a), n(b) {}
  bool hasNextValue() override { return i < n; }
  int64_t nextLongValue() override { if (i >= n) throw NoSuchElement(); return v[i++]; }
};
struct SeqDoubles : Doubles {
  const double* v; size_t n, i = 0;
  SeqDoubles(const double* a, size_t b) : v(a), n(b) {}
  bool hasNextValue() override { return i < n; }
  double nextDoubleValue() override { if (i >= n) throw NoSuchElement(); return v[i++]; }
};
int oracle_agg_long(int agg, const int64_t* v, size_t n, int64_t* out) {
  try { SeqLongs s(v, n); *out = runLong(agg, s); return 0; }
  catch (...) { return TSDBHIP_E_INVALID_ARG; }
}
int oracle_agg_double(int agg, const double* v, size_t n, double* out) {
  try { SeqDoubles s(v, n); *out = runDouble(agg, s); return 0; }
  catch (...) { return TSDBHIP_E_INVALID_ARG; }
}

// CompactionQueue.compact(row, compacted) for a batch of rows; host only.
// Same batch layout and output placement as tsdbhip_compact_rows
// (include/tsdbhip.h): row r's KVs are packed back to back in
// [row_qual_off[r], row_qual_off[r+1]) / [row_val_off[r], row_val_off[r+1]).
int oracle_compact_rows(const tsdbhip_rows_desc* d, tsdbhip_rows_out* out) {
  const uint64_t q0 = d->n_rows ? d->row_qual_off[0] : 0, v0 = d->n_rows ? d->row_val_off[0] : 0;
  uint64_t qu = 0, vu = 0, nc = 0;
  for (uint64_t r = 0; r < d->n_rows; r++) {
    std::vector<KeyValue> row;
    uint64_t qp = d->row_qual_off[r], vp = d->row_val_off[r];
    for (uint64_t k = d->row_kv_start[r]; k < d->row_kv_start[r + 1]; k++) {
      KeyValue kv;
      kv.base_time = 0;
      kv.qualifier = slice(d->qual_bytes, qp, d->kv_qual_len[k]);
      kv.value = slice(d->val_bytes, vp, d->kv_val_len[k]);
      kv.index = (int32_t)(k - d->row_kv_start[r]);
      qp += d->kv_qual_len[k];
      vp += d->kv_val_len[k];
      row.push_back(kv);
    }
    if (qp != d->row_qual_off[r + 1] || vp != d->row_val_off[r + 1]) return TSDBHIP_E_INVALID_ARG;
    CompactResult res;
    g_entered_complex = false;
    try {
      res = compact(row);
    } catch (JavaException& e) {
      res.status = e.code == TSDBHIP_E_OUT_OF_BOUNDS ? TSDBHIP_ROW_OOB : TSDBHIP_ROW_ERROR;
      res.qual.clear(); res.val.clear();
      res.write = false;  // the exception aborts the row: no put, no delete
      res.keep = -1;
    }
    const uint64_t oq = d->row_qual_off[r] - q0, ov = d->row_val_off[r] - v0 + r;
    if (oq + res.qual.size() > out->qual_capacity || ov + res.val.size() > out->val_capacity)
      return TSDBHIP_E_CAPACITY;
    if (g_entered_complex) nc++;
    out->row_status[r] = (uint8_t)res.status;
    out->row_qual_off[r] = oq;
    out->row_qual_len[r] = (uint32_t)res.qual.size();
    out->row_val_off[r] = ov;
    out->row_val_len[r] = (uint32_t)res.val.size();
    if (out->row_write) out->row_write[r] = res.write ? 1 : 0;
    if (out->row_keep_kv) out->row_keep_kv[r] = res.keep;
    if (!res.qual.empty()) std::memcpy(out->qual_bytes + oq, res.qual.data(), res.qual.size());
    if (!res.val.empty()) std::memcpy(out->val_bytes + ov, res.val.data(), res.val.size());
    qu = std::max<uint64_t>(qu, oq + res.qual.size());
    vu = std::max<uint64_t>(vu, ov + res.val.size());
  }
  (void)qu; (void)vu;
  out->qual_used = d->n_rows ? d->row_qual_off[d->n_rows] - q0 : 0;  // the extents, as tsdbhip_compact_rows
  out->val_used = d->n_rows ? d->row_val_off[d->n_rows] - v0 + d->n_rows : 0;
  out->n_complex = nc;
  return TSDBHIP_OK;
}


// ---------------------------------------------------------------------------
// Full-size checks of the benchmarked configurations (C1/C3/C3*): the
// synthetic SpanGroup of opentsdb_amd/synth.py regular() / the device
// generator tsdbhip_synth_generate, generated here shard by shard (span
// ranges of `shard_spans`), each shard run through the SGIterator above on
// its own thread, and the shard outputs combined in shard order. Valid only
// where the per-shard outputs combine into the whole group's: every shard
// must emit the same timestamps and types (aligned grids), and the
// aggregator must be sum (wrapping long add, or double add in shard order:
// the reference's order up to the rounding of the partial sums), min or
// max. Anything else returns TSDBHIP_E_INVALID_ARG.
static inline uint64_t smix64(uint64_t x) {  // splitmix64 (synth.py)
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t syn_hash3(uint64_t seed, uint64_t s, uint64_t i) {
  return smix64(smix64(seed ^ (s * 0xD1B54A32D192ED03ull)) ^ i);
}
// Rows of global series s: one compacted KeyValue per hour (trivialCompact
// layout: qualifiers, values, 0x00 when the row holds more than one cell).
static void syn_series(uint64_t seed, uint64_t s, uint32_t n_points, uint32_t t0, uint32_t step, uint32_t kind,
                       std::vector<KeyValue>& rows) {
  const uint32_t k = 3600 / step, w = kind == TSDBHIP_SYN_FLOAT32 ? 4 : 8;
  const uint32_t flags = kind == TSDBHIP_SYN_INT64_COUNTER ? 0x7 : (kind == TSDBHIP_SYN_FLOAT32 ? 0xB : 0xF);
  const uint64_t cbase = syn_hash3(seed, s, 0xFFFFFFFFull) >> 24;
  static const double INV_SD = 1.0 / 37837.0;
  rows.clear();
  for (uint32_t r = 0; (uint64_t)r * k < n_points; r++) {
    const uint32_t nc = std::min<uint32_t>(k, n_points - r * k);
    KeyValue kv;
    kv.base_time = t0 + r * 3600u;
    kv.qualifier.resize(2 * nc);
    kv.value.resize((size_t)nc * w + (nc > 1 ? 1 : 0));
    for (uint32_t c = 0; c < nc; c++) {
      const uint64_t i = (uint64_t)r * k + c;
      const uint32_t q = ((c * step) << 4) | flags;
      kv.qualifier[2 * c] = (uint8_t)(q >> 8);
      kv.qualifier[2 * c + 1] = (uint8_t)q;
      uint64_t be;
      const uint64_t h = syn_hash3(seed, s, i);
      if (kind == TSDBHIP_SYN_INT64_COUNTER) {
        be = cbase + 500ull * i + h % 500ull;
      } else {
        const int64_t sum = (int64_t)((h & 0xFFFF) + ((h >> 16) & 0xFFFF) + ((h >> 32) & 0xFFFF) +
                                      ((h >> 48) & 0xFFFF)) - 131070;
        const double v = 100.0 + (double)sum * INV_SD;
        if (kind == TSDBHIP_SYN_FLOAT32) {
          const float f = (float)v;
          uint32_t u;
          std::memcpy(&u, &f, 4);
          be = u;
        } else {
          std::memcpy(&be, &v, 8);
        }
      }
      for (uint32_t b = 0; b < w; b++) kv.value[(size_t)c * w + b] = (uint8_t)(be >> (8 * (w - 1 - b)));
    }
    rows.push_back(std::move(kv));
  }
}

struct ShardRes {
  int code = 0;
  uint64_t n_input = 0;
  std::vector<int64_t> ts, bits;
  std::vector<uint8_t> isint;
  // dev on the double path: the shard's Welford state per t (count, mean,
  // M2), the loop of Aggregators.java:219-238 run over the shard's values
  std::vector<int64_t> wn;
  std::vector<double> wmean, wm2;
};

static void run_regular_shard(uint64_t seed, uint32_t s0, uint32_t s1, uint32_t n_points, uint32_t t0, uint32_t step,
                              uint32_t kind, int64_t start, int64_t end, int agg, int rate, int32_t ds_interval,
                              int ds_agg, ShardRes& res) {
  try {
    std::vector<std::unique_ptr<Span>> spans(s1 - s0);
    std::vector<KeyValue> rows;
    for (uint32_t s = s0; s < s1; s++) {
      syn_series(seed, s, n_points, t0, step, kind, rows);
      spans[s - s0].reset(new Span());
      for (const KeyValue& kv : rows) spans[s - s0]->addRow(kv);
    }
    SpanGroup g;
    g.start_time = start;
    g.end_time = end;
    g.rate = rate != 0;
    g.aggregator = agg;
    g.downsampler = ds_interval > 0 ? ds_agg : -1;
    g.sample_interval = ds_interval;
    for (auto& sp : spans) g.add(sp.get());
    res.n_input = (uint64_t)g.aggregatedSize();
    SpanGroup::SGIterator it(&g);
    while (it.hasNext()) {
      it.next();
      res.ts.push_back(it.timestamp());
      const bool isint = it.isInteger();
      res.isint.push_back(isint ? 1 : 0);
      res.bits.push_back(isint ? it.longValue() : dbits(it.doubleValue()));
      if (agg == TSDBHIP_AGG_DEV && !isint) {  // the state behind doubleValue()'s sqrt
        it.pos = -1;
        double mean = it.nextDoubleValue(), m2 = 0;
        int64_t n = 1;
        while (it.hasNextValue()) {
          const double x = it.nextDoubleValue();
          n++;
          const double nm = mean + (x - mean) / (double)n;
          m2 += (x - mean) * (x - nm);
          mean = nm;
        }
        res.wn.push_back(n);
        res.wmean.push_back(mean);
        res.wm2.push_back(m2);
      }
    }
  } catch (JavaException& e) {
    res.code = e.code;
  }
}

int oracle_regular_sharded(uint64_t seed, uint32_t n_spans, uint32_t n_points, uint32_t t0, uint32_t step,
                           uint32_t kind, int64_t start, int64_t end, int agg, int rate, int32_t ds_interval,
                           int ds_agg, uint32_t shard_spans, int n_threads, tsdbhip_sg_out* out) {
  out->n_out = 0;
  out->n_input_points = 0;
  out->err_code = 0;
  out->err_index = -1;
  // (dev: double path only, i.e. rate or float series; the long dev truncates
  // a sequential Welford and admits no merge)
  const bool dev = agg == TSDBHIP_AGG_DEV;
  if (agg != TSDBHIP_AGG_SUM && agg != TSDBHIP_AGG_MIN && agg != TSDBHIP_AGG_MAX && !dev) return TSDBHIP_E_INVALID_ARG;
  if (dev && !rate && kind == TSDBHIP_SYN_INT64_COUNTER) return TSDBHIP_E_INVALID_ARG;
  if (!n_spans || !n_points || !step || 3600 % step || t0 % 3600 || kind > 2 || !shard_spans) return TSDBHIP_E_INVALID_ARG;
  const uint32_t n_shards = (n_spans + shard_spans - 1) / shard_spans;
  std::vector<ShardRes> res(n_shards);
  std::atomic<uint32_t> next{0};
  auto worker = [&]() {
    for (uint32_t sh; (sh = next.fetch_add(1)) < n_shards;)
      run_regular_shard(seed, sh * shard_spans, std::min(n_spans, (sh + 1) * shard_spans), n_points, t0, step,
                        kind, start, end, agg, rate, ds_interval, ds_agg, res[sh]);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < std::max(1, n_threads); t++) th.emplace_back(worker);
  for (auto& t : th) t.join();
  for (const ShardRes& r : res)
    if (r.code) return out->err_code = r.code;
  const ShardRes& a0 = res[0];
  const size_t T = a0.ts.size();
  if (T > out->capacity) return out->err_code = TSDBHIP_E_CAPACITY;
  for (size_t t = 0; t < T; t++) {
    out->ts[t] = a0.ts[t];
    out->is_int[t] = a0.isint[t];
    out->bits[t] = a0.bits[t];
  }
  uint64_t n_input = 0;
  std::vector<int64_t> wn;
  std::vector<double> wmean, wm2;
  if (dev) {
    if (a0.wn.size() != T) return out->err_code = TSDBHIP_E_INVALID_ARG;
    wn = a0.wn; wmean = a0.wmean; wm2 = a0.wm2;
  }
  for (uint32_t sh = 0; sh < n_shards; sh++) {
    const ShardRes& r = res[sh];
    n_input += r.n_input;
    if (sh == 0) continue;
    if (r.ts != a0.ts || r.isint != a0.isint) return out->err_code = TSDBHIP_E_INVALID_ARG;  // not aligned
    if (dev) {  // pairwise Welford merge in shard order (Chan et al.)
      for (size_t t = 0; t < T; t++) {
        const double na = (double)wn[t], nb = (double)r.wn[t], n = na + nb;
        const double delta = r.wmean[t] - wmean[t];
        wmean[t] += delta * (nb / n);
        wm2[t] += r.wm2[t] + delta * delta * (na * nb / n);
        wn[t] += r.wn[t];
        out->bits[t] = dbits(std::sqrt(wm2[t] / (double)wn[t]));
      }
      continue;
    }
    for (size_t t = 0; t < T; t++) {
      if (a0.isint[t]) {
        const int64_t x = r.bits[t], y = out->bits[t];
        out->bits[t] = agg == TSDBHIP_AGG_SUM ? ladd(y, x) : agg == TSDBHIP_AGG_MIN ? std::min(x, y) : std::max(x, y);
      } else {
        const double x = bitsd(r.bits[t]), y = bitsd(out->bits[t]);
        out->bits[t] = dbits(agg == TSDBHIP_AGG_SUM ? y + x : agg == TSDBHIP_AGG_MIN ? (x < y ? x : y) : (x > y ? x : y));
      }
    }
  }
  out->n_out = T;
  out->n_input_points = n_input;
  return TSDBHIP_OK;
}

}  // extern "C"
