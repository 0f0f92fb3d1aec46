//go:build mqmatch

// topics_gpu.go — reference-side binding of the MI355X engine (include/mqmatch.h).
//
// Drop this file (with go.mod's module github.com/xyzj/mqtt-server) next to topics.go and build
// with `-tags mqmatch` and CGO_ENABLED=1: it replaces the TopicsIndex of topics.go:349-698 with
// the same exported API, backed by the C-ABI. topics.go's TopicsIndex, NewTopicsIndex and the
// particle types must then be excluded from the build (`//go:build !mqmatch` on topics.go's
// index half); Subscribers, SelectShared, MergeSharedSelected, IsValidFilter, IsSharedFilter
// and the alias types stay as they are. server.go is unchanged: TopicsIndex.Retained keeps the
// method set server.go uses (Add, Get, GetAll, Len, Delete — server.go:980, 1717-1726), and
// its Add / Delete reach the engine. No Go toolchain exists in the build container, so this
// file is not compiled there; the same C-ABI calls, locking and id recycling are exercised by
// the C++ host mirror (csrc/host/topics_index.cpp, tests/cpp/test_topics_index.cpp).
package mqtt

/*
#cgo CFLAGS: -I${SRCDIR}/mqmatch/include
#cgo LDFLAGS: -L${SRCDIR}/mqmatch/lib -lmqmatch -Wl,-rpath,${SRCDIR}/mqmatch/lib
#include <stdlib.h>
#include "mqmatch.h"
*/
import "C"

import (
	"fmt"
	"log/slog"
	"math"
	"runtime"
	"strings"
	"sync"
	"sync/atomic"
	"time"
	"unsafe"

	"github.com/xyzj/mqtt-server/packets"
)

// noClient is an id no subscription uses: Unsubscribe for a client the index never saw still
// answers whether the filter's particle exists (topics.go:434-437).
const noClient = math.MaxUint32

// epochs tracks the match batches in flight. A batch's results may name any id that was in use
// when it began, so an id released at time r is reused only once every batch begun before r
// has ended.
type epochs struct {
	mu     sync.Mutex
	clock  uint64
	active map[uint64]int
}

func (e *epochs) begin() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.clock++
	e.active[e.clock]++
	return e.clock
}

func (e *epochs) end(t uint64) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.active[t]--; e.active[t] == 0 {
		delete(e.active, t)
	}
}

func (e *epochs) now() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.clock++
	return e.clock
}

func (e *epochs) oldest() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	m := uint64(math.MaxUint64)
	for t := range e.active {
		if t < m {
			m = t
		}
	}
	return m
}

// idTable maps strings (client IDs, filters, retained topics) to dense u32 ids, referenced by
// what uses them; an unreferenced id is released and later reused (epochs). Guarded by
// TopicsIndex.tables.
type idTable struct {
	ep   *epochs
	ids  map[string]uint32
	strs []string
	refs []uint32
	free []freeID // oldest release first
}

type freeID struct {
	id uint32
	at uint64
}

func newIDTable(ep *epochs) *idTable { return &idTable{ep: ep, ids: map[string]uint32{}} }

// intern returns the id of s, creating it unreferenced if new.
func (t *idTable) intern(s string) uint32 {
	if v, ok := t.ids[s]; ok {
		return v
	}
	var v uint32
	if len(t.free) > 0 && t.free[0].at < t.ep.oldest() {
		v = t.free[0].id
		t.free = t.free[1:]
		t.strs[v] = s
	} else {
		if len(t.strs) == noClient {
			panic("mqmatch: id space exhausted")
		}
		v = uint32(len(t.strs))
		t.strs = append(t.strs, s)
		t.refs = append(t.refs, 0)
	}
	t.ids[s] = v
	return v
}

func (t *idTable) find(s string) (uint32, bool) {
	v, ok := t.ids[s]
	return v, ok
}

func (t *idTable) ref(id uint32) { t.refs[id]++ }

// unref drops a reference; at zero the id is released at time `now`. tidy releases an id that
// was interned but never referenced.
func (t *idTable) unref(id uint32, now uint64) {
	t.refs[id]--
	t.tidy(id, now)
}

func (t *idTable) tidy(id uint32, now uint64) {
	if t.refs[id] != 0 {
		return
	}
	if v, ok := t.ids[t.strs[id]]; !ok || v != id {
		return // already released
	}
	delete(t.ids, t.strs[id]) // t.strs[id] stays readable for batches still in flight
	t.free = append(t.free, freeID{id, now})
}

type subKey struct {
	client uint32
	filter uint32
}

// RetainedPackets is TopicsIndex.Retained (topics.go:351): the reference's packets.Packets
// store, which server.go reads and sweeps directly (server.go:980, 1717-1726), wrapped so that
// entries added or deleted outside RetainMessage reach the engine as well — the expiry sweep's
// Delete drops the engine's entry and keeps the retain path (Q12); an Add makes the entry live
// again.
type RetainedPackets struct {
	*packets.Packets
	x *TopicsIndex
}

// Add (packets/packets.go:79-83). An engine error is logged and the store left as it was, so the
// store and the engine stay in step.
func (r *RetainedPackets) Add(id string, val packets.Packet) {
	x := r.x
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	h := x.topics.intern(id)
	x.tables.Unlock()
	p, n := cstr(id)
	if _, err := check(C.mq_retained_set(x.h, p, n, C.uint64_t(h), C.uint32_t(len(val.Payload)),
		boolU8(val.FixedHeader.Retain)), "mq_retained_set"); err != nil {
		x.tidyTopic(id)
		return
	}
	x.mapAdd(id, h, val)
}

// Delete (packets/packets.go:113-117).
func (r *RetainedPackets) Delete(id string) {
	x := r.x
	x.upd.Lock()
	defer x.upd.Unlock()
	p, n := cstr(id)
	if _, err := check(C.mq_retained_delete(x.h, p, n), "mq_retained_delete"); err != nil {
		return
	}
	x.mapDelete(id)
}

// TopicsIndex is the engine-backed index; same exported surface as topics.go:350-353.
//
// Locking: updates are serialised by upd (the engine serialises them as well); readers
// (Subscribers, Messages) never take it, and the engine's updates never wait for a reader's
// result (it copies what a live result may see, capi.cpp IndexLock), so a GPU round trip never
// waits for an update's lock nor an update for a reader. tables guards the id tables and the
// stored subscriptions.
//
// Errors: the reference's index cannot fail; the engine can (a lost device, MQ_EIO from a kernel
// guard). An update that fails is logged and answers false (nothing changed). A match batch that
// fails is tried again with backoff (retryDelays: about a third of a second in all), so a
// transient failure costs latency, not deliveries. A batch that fails every attempt has no answer
// to give — there is no CPU matching path — and it is not answered empty (round 6: that silently
// dropped the publish): SubscribersE / MessagesE return the error, and Subscribers / Messages,
// whose reference signatures cannot, hand it to EngineFailure (default: panic, the broker stops
// rather than acknowledge publishes it did not deliver; a broker may set it to log and carry on).
type TopicsIndex struct {
	Retained *RetainedPackets
	// EngineFailure is called when Subscribers or Messages cannot be answered (the batch failed
	// every attempt); nil: panic. op is "Subscribers" or "Messages", item the topic or filter.
	EngineFailure func(op, item string, err error)
	h        *C.mq_index
	upd      sync.Mutex
	tables   sync.RWMutex
	ep       *epochs
	// the batching stages Subscribers and Messages go through (started on first use)
	batcherOnce sync.Once
	batcher     *MatchBatcher
	msgOnce     sync.Once
	msgBatcher  *MessagesBatcher
	clients     *idTable
	filters     *idTable
	topics      *idTable // retained topic names: handle = topic id, referenced while in Retained
	stored      map[subKey]packets.Subscription
	inlineBy    map[subKey]InlineSubscription // (identifier, filter)
}

// NewTopicsIndex (topics.go:356-364). A broker that cannot open its engine cannot start, so this
// one failure panics, at start-up.
func NewTopicsIndex() *TopicsIndex {
	var h *C.mq_index
	cfg := C.mq_config{device: 0}
	if rc := C.mq_index_create(&cfg, &h); rc < 0 {
		panic(fmt.Sprintf("mq_index_create: %d %s", rc, C.GoString(C.mq_last_error())))
	}
	ep := &epochs{active: map[uint64]int{}}
	x := &TopicsIndex{
		h:        h,
		ep:       ep,
		clients:  newIDTable(ep),
		filters:  newIDTable(ep),
		topics:   newIDTable(ep),
		stored:   map[subKey]packets.Subscription{},
		inlineBy: map[subKey]InlineSubscription{},
	}
	x.Retained = &RetainedPackets{Packets: packets.NewPackets(), x: x}
	return x
}

func cstr(s string) (*C.char, C.uint32_t) {
	if len(s) == 0 {
		return nil, 0
	}
	return (*C.char)(unsafe.Pointer(unsafe.StringData(s))), C.uint32_t(len(s))
}

// EngineError is a failed engine call: the C-ABI's code (MQ_E*) and message.
type EngineError struct {
	Call string
	Code int
	Msg  string
}

func (e *EngineError) Error() string { return fmt.Sprintf("mqmatch: %s: %d %s", e.Call, e.Code, e.Msg) }

// check turns a C-ABI return code into an error, logged where it happens (the engine's message
// is per thread: read it now).
func check(rc C.int, what string) (C.int, error) {
	if rc >= 0 {
		return rc, nil
	}
	err := &EngineError{Call: what, Code: int(rc), Msg: C.GoString(C.mq_last_error())}
	slog.Error("mqmatch engine call failed", "call", what, "code", int(rc), "err", err.Msg)
	return rc, err
}

func boolU8(b bool) C.uint8_t {
	if b {
		return 1
	}
	return 0
}

// Subscribe (topics.go:401-419).
func (x *TopicsIndex) Subscribe(client string, sub packets.Subscription) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	cid, fid := x.clients.intern(client), x.filters.intern(sub.Filter)
	x.tables.Unlock()
	flags := C.uint8_t(0)
	if sub.NoLocal {
		flags |= C.MQ_SUB_NOLOCAL
	}
	if sub.RetainAsPublished {
		flags |= C.MQ_SUB_RAP
	}
	flags |= C.uint8_t(sub.RetainHandling&3) << C.MQ_SUB_RH_SHIFT
	p, n := cstr(sub.Filter)
	rc, err := check(C.mq_subscribe(x.h, p, n, C.uint32_t(cid), C.uint32_t(fid), C.uint8_t(sub.Qos), flags,
		C.int32_t(sub.Identifier)), "mq_subscribe")
	x.tables.Lock()
	defer x.tables.Unlock()
	k := subKey{cid, fid}
	if err != nil { // the interned ids go back if nothing references them
		now := x.ep.now()
		x.clients.tidy(cid, now)
		x.filters.tidy(fid, now)
		return false
	}
	if _, ok := x.stored[k]; !ok {
		x.clients.ref(cid)
		x.filters.ref(fid)
	}
	x.stored[k] = sub
	return rc == 1
}

// Unsubscribe (topics.go:423-448). An unknown client is looked up, never interned.
func (x *TopicsIndex) Unsubscribe(filter, client string) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.RLock()
	cid, okc := x.clients.find(client)
	fid, okf := x.filters.find(filter)
	x.tables.RUnlock()
	c := uint32(noClient)
	if okc {
		c = cid
	}
	p, n := cstr(filter)
	rc, err := check(C.mq_unsubscribe(x.h, p, n, C.uint32_t(c)), "mq_unsubscribe")
	if err != nil {
		return false
	}
	if okc && okf {
		x.tables.Lock()
		k := subKey{cid, fid}
		if _, ok := x.stored[k]; ok {
			delete(x.stored, k)
			now := x.ep.now()
			x.clients.unref(cid, now)
			x.filters.unref(fid, now)
		}
		x.tables.Unlock()
	}
	return rc == 1
}

// InlineSubscribe (topics.go:368-378).
func (x *TopicsIndex) InlineSubscribe(sub InlineSubscription) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	fid := x.filters.intern(sub.Filter)
	x.tables.Unlock()
	p, n := cstr(sub.Filter)
	rc, err := check(C.mq_inline_subscribe(x.h, p, n, C.int32_t(sub.Identifier), C.uint32_t(fid)), "mq_inline_subscribe")
	x.tables.Lock()
	defer x.tables.Unlock()
	if err != nil {
		x.filters.tidy(fid, x.ep.now())
		return false
	}
	k := subKey{uint32(sub.Identifier), fid}
	if _, ok := x.inlineBy[k]; !ok {
		x.filters.ref(fid)
	}
	x.inlineBy[k] = sub
	return rc == 1
}

// InlineUnsubscribe (topics.go:382-397).
func (x *TopicsIndex) InlineUnsubscribe(id int, filter string) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	p, n := cstr(filter)
	rc, err := check(C.mq_inline_unsubscribe(x.h, p, n, C.int32_t(id)), "mq_inline_unsubscribe")
	if err != nil {
		return false
	}
	x.tables.Lock()
	if fid, ok := x.filters.find(filter); ok {
		k := subKey{uint32(id), fid}
		if _, ok := x.inlineBy[k]; ok {
			delete(x.inlineBy, k)
			x.filters.unref(fid, x.ep.now())
		}
	}
	x.tables.Unlock()
	return rc == 1
}

// mapAdd / mapDelete keep the packet store and the topic id's reference together (upd held).
func (x *TopicsIndex) mapAdd(topic string, h uint32, pk packets.Packet) {
	if _, ok := x.Retained.Packets.Get(topic); !ok {
		x.tables.Lock()
		x.topics.ref(h)
		x.tables.Unlock()
	}
	x.Retained.Packets.Add(topic, pk)
}

func (x *TopicsIndex) mapDelete(topic string) {
	_, live := x.Retained.Packets.Get(topic)
	x.Retained.Packets.Delete(topic)
	x.tables.Lock()
	if h, ok := x.topics.find(topic); ok {
		if live {
			x.topics.unref(h, x.ep.now())
		} else {
			x.topics.tidy(h, x.ep.now())
		}
	}
	x.tables.Unlock()
}

// tidyTopic releases a topic id interned for an update that failed (upd held).
func (x *TopicsIndex) tidyTopic(topic string) {
	x.tables.Lock()
	if h, ok := x.topics.find(topic); ok {
		x.topics.tidy(h, x.ep.now())
	}
	x.tables.Unlock()
}

// RetainMessage (topics.go:453-476). The Go packets map stays the store of packets and answers
// the -1 case from the replaced packet as the reference does; the engine keeps the retain paths
// and liveness. A failed engine call changes nothing and answers 0.
func (x *TopicsIndex) RetainMessage(pk packets.Packet) int64 {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	h := x.topics.intern(pk.TopicName)
	x.tables.Unlock()
	p, n := cstr(pk.TopicName)
	var out C.int64_t
	if _, err := check(C.mq_retain_message(x.h, p, n, C.uint64_t(h), C.uint32_t(len(pk.Payload)),
		boolU8(pk.FixedHeader.Retain), &out), "mq_retain_message"); err != nil {
		x.tidyTopic(pk.TopicName)
		return 0
	}
	if len(pk.Payload) > 0 {
		x.mapAdd(pk.TopicName, h, pk)
		return 1
	}
	var r int64
	if pke, ok := x.Retained.Packets.Get(pk.TopicName); ok && len(pke.Payload) > 0 && pke.FixedHeader.Retain {
		r = -1
	}
	x.mapDelete(pk.TopicName)
	return r
}

// pack concatenates strings for the engine: offsets, plus the 16 readable padding bytes the
// C-ABI asks of an input buffer (include/mqmatch.h).
func pack(items []string) ([]byte, []uint64) {
	offs := make([]uint64, len(items)+1)
	total := 0
	for _, s := range items {
		total += len(s)
	}
	buf := make([]byte, 0, total+16)
	for i, s := range items {
		buf = append(buf, s...)
		offs[i+1] = uint64(len(buf))
	}
	buf = append(buf, make([]byte, 16)...)
	return buf, offs
}

// Messages (topics.go:525-579). A filter without wildcards is the packet store's own lookup,
// as in the reference (topics.go:539-544); the others go through the index's Messages batching
// stage: publishRetainedToClient calls Messages once per filter of every SUBSCRIBE, from every
// connection goroutine (server.go:1115-1133), so the wildcard filters of many goroutines share
// one engine call. An engine failure answers no retained messages (logged).
func (x *TopicsIndex) Messages(filter string) []packets.Packet {
	if len(filter) == 0 || x.Retained.Len() == 0 {
		return []packets.Packet{}
	}
	if !strings.ContainsRune(filter, '#') && !strings.ContainsRune(filter, '+') {
		pks := []packets.Packet{}
		if pk, ok := x.Retained.Get(filter); ok {
			pks = append(pks, pk)
		}
		return pks
	}
	pks, err := x.MessagesE(filter)
	if err != nil {
		x.engineFailed("Messages", filter, err)
		return []packets.Packet{}
	}
	return pks
}

// MessagesE is Messages with the engine's failure returned (wildcard filters: a batch that failed
// every attempt).
func (x *TopicsIndex) MessagesE(filter string) ([]packets.Packet, error) {
	if len(filter) == 0 || x.Retained.Len() == 0 ||
		(!strings.ContainsRune(filter, '#') && !strings.ContainsRune(filter, '+')) {
		return x.Messages(filter), nil
	}
	x.msgOnce.Do(func() { x.msgBatcher = NewMessagesBatcher(x, DefaultMaxBatch, DefaultMinFill, DefaultMaxDelay) })
	return x.msgBatcher.get(filter)
}

// MessagesBatch answers Messages for many filters with one engine call.
func (x *TopicsIndex) MessagesBatch(filters []string) ([][]packets.Packet, error) {
	v, err := x.matchMessages(filters)
	if err != nil {
		return nil, err
	}
	v.refs.Store(1)
	out := make([][]packets.Packet, len(filters))
	for i := range filters {
		out[i] = v.get(i)
	}
	v.release()
	return out, nil
}

// msgView is one mq_messages_runs_batch result, shared by the callers whose filters it matched:
// each filter's handles as runs of the retained image's handle array (round 6: the engine no longer
// copies every handle out; the runs are expanded here, on the caller's goroutine).
type msgView struct {
	x       *TopicsIndex
	r       *C.mq_msg_runs_result
	stamp   uint64
	refs    atomic.Int32
	runBase []C.uint64_t
	nRuns   []C.uint32_t
	count   []C.uint32_t
	runs    []C.mq_msg_run
	handle  []uint64
}

func (x *TopicsIndex) matchMessages(filters []string) (*msgView, error) {
	stamp := x.ep.begin()
	buf, offs := pack(filters)
	var r *C.mq_msg_runs_result
	if _, err := check(C.mq_messages_runs_batch(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), C.uint32_t(len(filters)), &r),
		"mq_messages_runs_batch"); err != nil {
		x.ep.end(stamp)
		return nil, err
	}
	v := &msgView{x: x, r: r, stamp: stamp}
	n := int(r.n_filters)
	v.runBase = unsafe.Slice(r.run_base, n)
	v.nRuns = unsafe.Slice(r.n_runs, n)
	v.count = unsafe.Slice(r.count, n)
	v.runs = unsafe.Slice(r.runs, int(r.n_runs_total))
	v.handle = unsafe.Slice((*uint64)(unsafe.Pointer(r.handles)), int(r.n_handles))
	return v, nil
}

// get expands filter i's runs and resolves the handles to packets, on the caller's goroutine.
func (v *msgView) get(i int) []packets.Packet {
	topics := make([]string, 0, int(v.count[i]))
	rs := v.runs[v.runBase[i] : v.runBase[i]+C.uint64_t(v.nRuns[i])]
	v.x.tables.RLock()
	for _, run := range rs {
		for _, h := range v.handle[run.first : run.first+run.count] {
			topics = append(topics, v.x.topics.strs[h])
		}
	}
	v.x.tables.RUnlock()
	pks := []packets.Packet{}
	for _, t := range topics {
		if pk, ok := v.x.Retained.Get(t); ok {
			pks = append(pks, pk)
		}
	}
	return pks
}

func (v *msgView) release() {
	if v.refs.Add(-1) == 0 {
		C.mq_result_free(unsafe.Pointer(v.r))
		v.x.ep.end(v.stamp)
	}
}

// Subscribers (topics.go:583-590). publishToSubscribers calls it once per publish from every
// connection goroutine (server.go:1000); the call goes through the index's batching stage, which
// matches the topics of many goroutines with one engine call (MatchBatcher below), so server.go
// keeps calling Subscribers unchanged. The maps are built here, on the caller's goroutine, from the
// batch's shared span result, as the reference builds them on every connection goroutine.
func (x *TopicsIndex) Subscribers(topic string) *Subscribers {
	s, err := x.SubscribersE(topic)
	if err != nil {
		x.engineFailed("Subscribers", topic, err)
		return emptySubscribers()
	}
	return s
}

// SubscribersE is Subscribers with the engine's failure returned (a batch that failed every
// attempt) — for a caller that can refuse the publish instead (INTEGRATION.md §3).
func (x *TopicsIndex) SubscribersE(topic string) (*Subscribers, error) {
	x.batcherOnce.Do(func() { x.batcher = NewMatchBatcher(x, DefaultMaxBatch, DefaultMinFill, DefaultMaxDelay) })
	return x.batcher.get(topic)
}

// engineFailed: Subscribers / Messages could not be answered (EngineFailure, default panic).
func (x *TopicsIndex) engineFailed(op, item string, err error) {
	if x.EngineFailure != nil {
		x.EngineFailure(op, item, err)
		return
	}
	panic(fmt.Errorf("mqmatch: %s(%q) failed on every attempt: %w", op, item, err))
}

func emptySubscribers() *Subscribers {
	return &Subscribers{
		Shared:              map[string]map[string]packets.Subscription{},
		SharedSelected:      map[string]packets.Subscription{},
		Subscriptions:       map[string]packets.Subscription{},
		InlineSubscriptions: map[int]InlineSubscription{},
	}
}

// The batching stages' defaults (SURVEY.md §8f.1; DESIGN.md §7 has the measured batch latency).
const (
	DefaultMaxBatch = 16384                  // items per engine call at most
	DefaultMinFill  = 1024                   // under load, a batch with fewer items waits for more ...
	DefaultMaxDelay = 200 * time.Microsecond // ... up to this long
)

// batchView is one engine call's result, shared by the callers whose items it matched: each
// caller builds its own answer from it (get, on the caller's goroutine), then releases it; the
// last release frees the engine's result.
type batchView[T any] interface {
	get(i int) T
	release()
	setRefs(n int) // the number of releases to come (set before any caller gets the view)
}

type batchReq[T any] struct {
	item  string
	reply chan batchReply[T]
}

type batchReply[T any] struct {
	view batchView[T]
	i    int
	err  error
}

// batcher is a batching stage (SURVEY.md §8f.1): caller goroutines hand their item to one loop
// goroutine per stage and wait for their reply; the loop takes every request queued when the
// previous batch is done — under load, what arrived while it was matched — and matches the batch
// with one engine call (run). When the previous batch held more than one request (there is
// concurrent load), a batch with fewer than minFill items first waits up to maxDelay for more; a
// lone request on an idle stage is matched at once. A failed engine call is tried again after each
// of retryDelays; if every attempt fails, every caller of the batch gets the error (logged by
// check), never an empty answer.
type batcher[T any] struct {
	run      func(items []string) (batchView[T], error)
	in       chan batchReq[T]
	maxBatch int
	minFill  int
	maxDelay time.Duration
	done     chan struct{}
	replies  sync.Pool
	failed   atomic.Uint64 // batches whose callers got the error
}

// retryDelays: the waits before a failed batch's further attempts (about a third of a second).
var retryDelays = []time.Duration{0, time.Millisecond, 4 * time.Millisecond, 16 * time.Millisecond,
	64 * time.Millisecond, 256 * time.Millisecond}

func newBatcher[T any](run func([]string) (batchView[T], error), maxBatch, minFill int,
	maxDelay time.Duration) *batcher[T] {
	if maxBatch <= 0 {
		maxBatch = DefaultMaxBatch
	}
	if minFill <= 0 || minFill > maxBatch {
		minFill = maxBatch
	}
	b := &batcher[T]{run: run, in: make(chan batchReq[T], 4*maxBatch), maxBatch: maxBatch,
		minFill: minFill, maxDelay: maxDelay, done: make(chan struct{})}
	b.replies.New = func() any { return make(chan batchReply[T], 1) }
	go b.loop()
	return b
}

// get enqueues item, waits for the batch it joins and builds its answer (or returns the batch's
// error: every attempt failed).
func (b *batcher[T]) get(item string) (T, error) {
	r := b.replies.Get().(chan batchReply[T])
	b.in <- batchReq[T]{item, r}
	rep := <-r
	b.replies.Put(r)
	if rep.err != nil {
		var zero T
		return zero, rep.err
	}
	v := rep.view.get(rep.i)
	rep.view.release()
	return v, nil
}

// Failed counts the batches whose callers got the error.
func (b *batcher[T]) Failed() uint64 { return b.failed.Load() }

// Close matches what is queued and stops the loop; no get may follow.
func (b *batcher[T]) Close() {
	close(b.in)
	<-b.done
}

func (b *batcher[T]) loop() {
	// The loop stays on one OS thread: the HIP runtime sets up per-thread state on a thread's first
	// call (~10 ms), and a goroutine that moved to a fresh thread would pay it again inside a match,
	// under the index's lock (the engine also warms a new calling thread before taking the lock:
	// mq_thread_warm, INTEGRATION.md §3).
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	defer close(b.done)
	batch := make([]batchReq[T], 0, b.maxBatch)
	items := make([]string, 0, b.maxBatch)
	timer := time.NewTimer(time.Hour)
	timer.Stop()
	last := 0 // the previous batch's size
	for {
		r, ok := <-b.in
		if !ok {
			return
		}
		batch = append(batch[:0], r)
		open := true
	drain: // everything queued now, without waiting
		for len(batch) < b.maxBatch {
			select {
			case r, ok := <-b.in:
				if !ok {
					open = false
					break drain
				}
				batch = append(batch, r)
			default:
				break drain
			}
		}
		if open && last > 1 && len(batch) < b.minFill && b.maxDelay > 0 { // under load: wait a little for more
			timer.Reset(b.maxDelay)
		wait:
			for len(batch) < b.maxBatch {
				select {
				case r, ok := <-b.in:
					if !ok {
						break wait
					}
					batch = append(batch, r)
					if len(batch) >= b.minFill {
						break wait
					}
				case <-timer.C:
					break wait
				}
			}
			timer.Stop()
		}
		last = len(batch)
		items = items[:0]
		for _, r := range batch {
			items = append(items, r.item)
		}
		v, err := b.call(items)
		for k := 0; err != nil && k < len(retryDelays); k++ { // a transient failure costs retries, not the batch
			time.Sleep(retryDelays[k])
			v, err = b.call(items)
		}
		if err != nil {
			b.failed.Add(1)
			for _, r := range batch {
				r.reply <- batchReply[T]{err: err}
			}
		} else {
			for i, r := range batch {
				r.reply <- batchReply[T]{view: v, i: i}
			}
		}
		clear(batch) // drop the references to the replies
	}
}

// call runs the engine call with the view's reference count set before any caller can release
// it; a panic in it (a bug, not an engine error) becomes this batch's error.
func (b *batcher[T]) call(items []string) (v batchView[T], err error) {
	defer func() {
		if p := recover(); p != nil {
			v, err = nil, fmt.Errorf("mqmatch: batch of %d: %v", len(items), p)
			slog.Error("mqmatch batch panicked", "items", len(items), "panic", p)
		}
	}()
	v, err = b.run(items)
	if err == nil {
		v.setRefs(len(items))
	}
	return v, err
}

// MatchBatcher is the Subscribers stage; MessagesBatcher the Messages stage.
type (
	MatchBatcher    = batcher[*Subscribers]
	MessagesBatcher = batcher[[]packets.Packet]
)

// NewMatchBatcher starts a Subscribers batching stage over x.
func NewMatchBatcher(x *TopicsIndex, maxBatch, minFill int, maxDelay time.Duration) *MatchBatcher {
	run := func(items []string) (batchView[*Subscribers], error) {
		v, err := x.matchSpans(items)
		if err != nil {
			return nil, err
		}
		return v, nil
	}
	return newBatcher[*Subscribers](run, maxBatch, minFill, maxDelay)
}

// NewMessagesBatcher starts a Messages batching stage over x (wildcard filters only).
func NewMessagesBatcher(x *TopicsIndex, maxBatch, minFill int, maxDelay time.Duration) *MessagesBatcher {
	run := func(items []string) (batchView[[]packets.Packet], error) {
		v, err := x.matchMessages(items)
		if err != nil {
			return nil, err
		}
		return v, nil
	}
	return newBatcher[[]packets.Packet](run, maxBatch, minFill, maxDelay)
}

func (v *msgView) setRefs(n int)  { v.refs.Store(int32(n)) }
func (v *spanView) setRefs(n int) { v.refs.Store(int32(n)) }

// spanView is one mq_match_spans result (span format: the index's own records plus patches, per
// topic or shared by a merge set, include/mqmatch.h), shared by the callers whose topics it
// matched. The host records it points into stay as they were at the match until it is freed
// (the engine copies what it changes), and the ids it names stay reserved until then (epochs);
// a subscription removed between the match and a caller's get is rebuilt from its record.
type spanView struct {
	x          *TopicsIndex
	r          *C.mq_span_result
	stamp      uint64
	refs       atomic.Int32
	ts         []C.mq_topic_spans
	spans      []C.mq_span
	patches    []C.mq_patch
	setPatches []C.mq_patch
	mergeRows  []C.uint32_t
	mergeBase  []C.uint32_t
	inl        []C.mq_inline_row
	picked     []C.mq_shared_row
	subPool    []C.mq_client_row
	shrPool    []C.mq_shared_row
	pickedOnly bool
	codes      bool     // 4-byte patch codes (MQ_SPANS_PATCH_CODES): patchCodes / setCodes instead
	patchCodes []uint32 // of patches / setPatches
	setCodes   []uint32
}

func (x *TopicsIndex) matchSpans(topics []string) (*spanView, error) {
	stamp := x.ep.begin()
	buf, offs := pack(topics)
	var r *C.mq_span_result
	if _, err := check(C.mq_match_spans(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), C.uint32_t(len(topics)), &r),
		"mq_match_spans"); err != nil {
		x.ep.end(stamp)
		return nil, err
	}
	v := &spanView{x: x, r: r, stamp: stamp}
	v.ts = unsafe.Slice(r.topics, int(r.n_topics))
	v.spans = unsafe.Slice(r.spans, int(r.n_spans))
	v.codes = r.flags&C.MQ_SPANS_PATCH_CODES != 0
	// merge-set patches (MQ_TOPIC_SET_PATCHES): row x<<MQ_SET_ROW_BITS|k (codes:
	// x<<MQ_CODE_SET_ROW_BITS|k) is record k of the topic's x-th may-merge particle, whose first
	// row is merge_rows[merge_row_base[topic]+x]
	if v.codes {
		v.patchCodes = unsafe.Slice((*uint32)(unsafe.Pointer(r.patches)), int(r.n_patches))
		v.setCodes = unsafe.Slice((*uint32)(unsafe.Pointer(r.set_patches)), int(r.n_set_patches))
	} else {
		v.patches = unsafe.Slice(r.patches, int(r.n_patches))
		v.setPatches = unsafe.Slice(r.set_patches, int(r.n_set_patches))
	}
	v.mergeRows = unsafe.Slice(r.merge_rows, int(r.n_merge_rows))
	if r.merge_row_base != nil {
		v.mergeBase = unsafe.Slice(r.merge_row_base, int(r.n_topics))
	}
	v.inl = unsafe.Slice(r.inline_rows, int(r.n_inline_rows))
	v.picked = unsafe.Slice(r.picked_rows, int(r.n_picked_rows))
	v.subPool = unsafe.Slice(r.sub_pool, int(r.sub_pool_len))
	v.shrPool = unsafe.Slice(r.shared_pool, int(r.shared_pool_len))
	v.pickedOnly = r.flags&C.MQ_SPANS_PICKED != 0
	return v, nil
}

// patchOp marks a patch code's op in the patched map (MQ_PATCH_OP); patchApply is mq_patch_apply:
// op 1..6 the merge base with Qos (op-1)%3 and NoLocal (op-1)/3, op 7 a later match.
const patchOp = uint32(C.MQ_PATCH_OP)

func patchApply(p, meta uint32, ident int32) uint32 {
	if p&patchOp == 0 {
		return p
	}
	op := p & 7
	if op == 7 {
		if ident > 0 {
			return meta | C.MQ_ROW_IDENT
		}
		return meta | C.MQ_ROW_DROP
	}
	meta &^= C.MQ_META_QOS_MASK | C.MQ_META_NOLOCAL
	meta |= (op - 1) % 3
	if (op-1)/3 != 0 {
		meta |= C.MQ_META_NOLOCAL
	}
	return meta
}

func (v *spanView) release() {
	if v.refs.Add(-1) == 0 {
		C.mq_result_free(unsafe.Pointer(v.r))
		v.x.ep.end(v.stamp)
	}
}

// SubscribersBatch matches many topics in one engine call and builds their Subscribers here.
func (x *TopicsIndex) SubscribersBatch(topics []string) ([]*Subscribers, error) {
	v, err := x.matchSpans(topics)
	if err != nil {
		return nil, err
	}
	v.refs.Store(1)
	out := make([]*Subscribers, len(topics))
	for i := range topics {
		out[i] = v.get(i)
	}
	v.release()
	return out, nil
}

// get builds topic i's Subscribers (topics.go:583-590, Subscription.Merge packets.go:254-274 as
// the engine resolved it), on the caller's goroutine.
func (v *spanView) get(i int) *Subscribers {
	x := v.x
	x.tables.RLock()
	defer x.tables.RUnlock()
	stored := func(c, f uint32, ident int32, meta uint32) packets.Subscription {
		if s, ok := x.stored[subKey{c, f}]; ok {
			return s
		}
		return packets.Subscription{Filter: x.filters.strs[f], Identifier: int(ident), Qos: byte(meta & C.MQ_META_QOS_MASK)}
	}
	t := v.ts[i]
	s := emptySubscribers()
	var patched map[uint32]uint32 // topic row -> meta, or patchOp | op (a patch code)
	if t.n_patches > 0 {
		patched = make(map[uint32]uint32, int(t.n_patches))
	}
	lo, hi := t.patch_base, t.patch_base+C.uint64_t(t.n_patches)
	set := t.flags&C.MQ_TOPIC_SET_PATCHES != 0
	var mr []C.uint32_t
	if set {
		mr = v.mergeRows[v.mergeBase[i]:]
	}
	topicRow := func(row, bits uint32) uint32 { // a set patch's row, through the topic's merge rows
		if !set {
			return row
		}
		return uint32(mr[row>>bits]) + row&(1<<bits-1)
	}
	switch {
	case v.codes && set:
		for _, c := range v.setCodes[lo:hi] {
			patched[topicRow(c>>3, C.MQ_CODE_SET_ROW_BITS)] = patchOp | c&7
		}
	case v.codes:
		for _, c := range v.patchCodes[lo:hi] {
			patched[c>>3] = patchOp | c&7
		}
	case set:
		for _, pt := range v.setPatches[lo:hi] {
			patched[topicRow(uint32(pt.row), C.MQ_SET_ROW_BITS)] = uint32(pt.meta)
		}
	default:
		for _, pt := range v.patches[lo:hi] {
			patched[uint32(pt.row)] = uint32(pt.meta)
		}
	}
	addShared := func(sr C.mq_shared_row) {
		f, c := x.filters.strs[sr.filter_id], x.clients.strs[sr.client_id]
		if _, ok := s.Shared[f]; !ok {
			s.Shared[f] = map[string]packets.Subscription{}
		}
		s.Shared[f][c] = stored(uint32(sr.client_id), uint32(sr.filter_id), 0, 0)
	}
	// records in gather order: a client's client row precedes its ident rows
	row := uint32(0)
	for _, sp := range v.spans[t.span_base : t.span_base+C.uint64_t(t.n_spans)] {
		for _, cr := range v.subPool[sp.sub_off : sp.sub_off+sp.n_sub] {
			meta := uint32(cr.meta)
			if m, ok := patched[row]; ok {
				meta = patchApply(m, meta, int32(cr.identifier))
			}
			row++
			switch meta & C.MQ_ROW_KIND_MASK {
			case 0: // client row: the merged Subscription
				base := stored(uint32(cr.client_id), uint32(cr.filter_id), int32(cr.identifier), meta)
				base.Qos = byte(meta & C.MQ_META_QOS_MASK)
				base.NoLocal = meta&C.MQ_META_NOLOCAL != 0
				base.Identifiers = map[string]int{base.Filter: base.Identifier}
				s.Subscriptions[x.clients.strs[cr.client_id]] = base
			case C.MQ_ROW_IDENT: // a further Identifiers entry of that client
				sub := s.Subscriptions[x.clients.strs[cr.client_id]]
				sub.Identifiers[x.filters.strs[cr.filter_id]] = int(cr.identifier)
			}
		}
		if !v.pickedOnly {
			for _, sr := range v.shrPool[sp.shr_off : sp.shr_off+sp.n_shr] {
				addShared(sr)
			}
		}
	}
	if v.pickedOnly {
		for _, sr := range v.picked[t.picked_base : t.picked_base+C.uint64_t(t.n_shared)] {
			addShared(sr)
		}
	}
	for _, lr := range v.inl[t.inline_base : t.inline_base+C.uint64_t(t.n_inline)] {
		in, ok := x.inlineBy[subKey{uint32(lr.identifier), uint32(lr.filter_id)}]
		if !ok { // unsubscribed since the match
			in = InlineSubscription{Subscription: packets.Subscription{Filter: x.filters.strs[lr.filter_id],
				Identifier: int(lr.identifier)}}
		}
		s.InlineSubscriptions[int(lr.identifier)] = in
	}
	return s
}
