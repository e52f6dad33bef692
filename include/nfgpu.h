/* nfgpu.h — C-ABI boundary of the MI355X-native NoahGameFrame per-tick entity
 * update path (heartbeat scan -> property/record mutation -> dirty diff ->
 * scene-group fan-out).  Plain pointers and sizes only.
 *
 * Every entry point names the reference interface it replaces.  Reference
 * paths are relative to flyish/NoahGameFrame:
 *   KM  = NFComm/NFKernelPlugin/NFCKernelModule.cpp
 *   SM  = NFComm/NFKernelPlugin/NFCScheduleModule.cpp
 *   AOI = NFComm/NFKernelPlugin/NFCSceneAOIModule.cpp
 *   PR  = NFComm/NFCore/NFCProperty.cpp
 *   RC  = NFComm/NFCore/NFCRecord.cpp
 *
 * Entities are addressed by NFGUID (head, data) exactly like NFIKernelModule.
 * Outputs address entities by "object index" = creation order in this world
 * (nfk_create_objects call order), which the host maps back to NFGUID.
 */
#ifndef NFGPU_H
#define NFGPU_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (every call returns one; nothing fails silently) ---- */
#define NFK_OK 0
#define NFK_ERR_ARG (-1)       /* bad argument / schema violation */
#define NFK_ERR_HIP (-2)       /* HIP runtime error (no GPU, OOM, launch failure) */
#define NFK_ERR_STATE (-3)     /* call out of order (e.g. execute before commit) */
#define NFK_ERR_CAPACITY (-4)  /* entity / event / message capacity exceeded */
#define NFK_ERR_TOUCH (-5)     /* > NFK_MAX_TOUCH distinct properties written per entity per tick */
#define NFK_ERR_DEVICE (-6)    /* device-side error word set (bounded spin expired) */
#define NFK_ERR_NOTFOUND (-7)  /* GUID not present */

#define NFK_MAX_INT_PROPS 64
#define NFK_MAX_FLT_PROPS 64
#define NFK_MAX_OBJ_PROPS 32 /* object (NFGUID) properties; n_int + n_flt + n_obj <= NFK_MAX_PROPS */
#define NFK_MAX_PROPS 128
#define NFK_MAX_CLASSES 16 /* class id 15 is reserved (marks a free slot on the device) */
#define NFK_MAX_KINDS 32
#define NFK_MAX_OPS 8     /* ops per heartbeat program */
#define NFK_MAX_REC_OPS 4 /* record ops across all programs (distinct record columns) */
#define NFK_MAX_RECORDS 8
#define NFK_MAX_REC_ROWS 64
#define NFK_MAX_REC_COLS 16
#define NFK_MAX_TOUCH 12

/* property / record visibility flags, NFIProperty::GetPublic/GetPrivate/GetUpload */
#define NFK_PUBLIC 1
#define NFK_PRIVATE 2
#define NFK_UPLOAD 4

/* Heartbeat effect ops.  A reference game registers arbitrary C++ functors
 * with NFIScheduleModule::AddSchedule (SM:218); on the device a heartbeat
 * kind carries a program of these ops, each one a Get + Set through the
 * reference's change predicates (PR:254 SetInt, PR:295 SetFloat, RC:182
 * SetInt, RC:243 SetFloat).
 *   IADD_CLAMP  dst(int) = clamp(dst + A, LO, HI)        A/LO/HI imm or prop
 *   FLERP       dst(f64) = dst + (prop[a] - dst) * f64(b) (no FMA contraction)
 *   FAFFINE     dst(f64) = dst * f64(a) + f64(b)
 *   RIADD_CLAMP record cell(int) = clamp(cell + a, b, c) for every used row
 *   RFAFFINE    record cell(f64) = cell * f64(a) + f64(b) for every used row
 *   ISET        dst(int) = A                                  A imm or prop (NFK_A_PROP)
 *   FSET        dst(f64) = A                                  A f64(a) or f64 prop (NFK_A_PROP)
 * clamp(v, lo, hi): v < lo -> lo; then v > hi -> hi.  Integer adds wrap.
 * Record ops: dst = (rec << 8) | col.
 * NFK_GUARD (property ops only): the op runs only when int property (guard & 0xFFFF), as the
 * program has left it so far, compares to 0 as NFK_GUARD_* in (guard >> 16) & 3 says — a functor's
 * `if (GetPropertyInt(self, g) > 0) SetProperty...(...)`.  With NFK_GUARD_PROP in guard it compares
 * to int property (guard >> 19) instead of 0 (both as the program has left them):
 * `if (GetPropertyInt(self, g) > GetPropertyInt(self, h)) ...`.  Without it, bits 19..31 hold a
 * signed constant K in [-4096, 4095] (NFK_GUARD_K; 0 by default) that g is compared to instead:
 * `if (GetPropertyInt(self, g) > 10) ...` (>= K and < K are > K-1 and <= K-1). */
enum {
    NFK_OP_NOP = 0,
    NFK_OP_IADD_CLAMP = 1,
    NFK_OP_FLERP = 2,
    NFK_OP_FAFFINE = 3,
    NFK_OP_RIADD_CLAMP = 4,
    NFK_OP_RFAFFINE = 5,
    NFK_OP_ISET = 6,
    NFK_OP_FSET = 7
};
#define NFK_A_PROP 1
#define NFK_LO_PROP 2
#define NFK_HI_PROP 4
#define NFK_GUARD 8
#define NFK_GUARD_GT0 0 /* g > 0 */
#define NFK_GUARD_LE0 1 /* g <= 0 */
#define NFK_GUARD_NE0 2 /* g != 0 */
#define NFK_GUARD_EQ0 3 /* g == 0 */
#define NFK_GUARD_PROP (1u << 18) /* compare g to int property guard >> 19 (< 8192) instead of 0 */
#define NFK_GUARD_K(k) (((uint32_t)(k) & 0x1FFFu) << 19) /* compare g to the constant k (no NFK_GUARD_PROP) */
#define NFK_GUARD_KVAL(guard) ((int32_t)(guard) >> 19)   /* the constant of a guard word without NFK_GUARD_PROP */
#define NFK_GUARD_KMIN (-4096)
#define NFK_GUARD_KMAX 4095

typedef struct nfk_op {
    uint8_t code;
    uint8_t flags;
    uint16_t dst;
    uint32_t guard; /* with NFK_GUARD: property id | NFK_GUARD_* << 16 [| NFK_GUARD_PROP | h << 19 or | NFK_GUARD_K(k)]; else 0 */
    int64_t a, b, c;
} nfk_op; /* 32 bytes */

typedef struct nfk_config {
    int32_t capacity;     /* max entities resident on this GPU */
    int32_t n_int;        /* int64 property columns, prop ids [0, n_int) */
    int32_t n_flt;        /* f64 property columns, prop ids [n_int, n_int+n_flt) */
    int32_t n_class;      /* classes (NFIClassModule), flags per class */
    int32_t n_kind;       /* heartbeat kinds; id order MUST equal lexical name order */
    int32_t n_rec;        /* records */
    int64_t msg_capacity; /* fan-out messages per tick (0 = 32 x capacity) */
    void* stream;         /* hipStream_t to launch on, NULL = library-owned stream */
    int32_t slack_per_256; /* free slots kept per 256 members of a scene group for arrivals
                              (SwitchScene / imports) without a full re-layout:
                              0 = default 16, < 0 = none */
    int32_t n_obj;        /* object (NFGUID) property columns, prop ids [n_int+n_flt, +n_obj):
                             16 bytes per entity (data, head), TDATA_OBJECT (NFIDataList.h) */
} nfk_config;

typedef struct nfk_summary {
    int64_t n_entities;
    int64_t n_prop_events;  /* coalesced dirty (entity, property) pairs this tick */
    int64_t n_rec_events;   /* coalesced dirty (entity, record, row, col) cells */
    int64_t n_fired;        /* heartbeat callbacks fired (NFCScheduleElement::DoHeartBeatEvent) */
    int64_t n_msgs;         /* fan-out messages (event x recipient) */
    int64_t alg_bytes_tick; /* algorithmic HBM bytes of the tick kernel this tick */
    int64_t alg_bytes_rec;  /* ... of the record kernel */
    int64_t alg_bytes_fan;  /* ... of the fan-out kernel */
    int32_t device_error;   /* nonzero: device error word */
    int32_t tick;           /* ticks executed */
} nfk_summary;

/* Device-resident outputs of the last tick (valid until the next execute).
 *
 * Outputs are TILE-STAGED: property events and fired heartbeats are grouped by 256-slot tile
 * (tile t = slots [256t, 256t+256) in (scene, group, guid) order), record events by 64-slot
 * record tile.  The i-th output of tile t sits at index t * <x>_tile_cap + i, for
 * i < <x>_base[t+1] - <x>_base[t]; its rank in the global order is <x>_base[t] + i.  Walking
 * tiles in order and each tile's entries in order gives exactly the reference order:
 *   property events  (scene, group, guid, prop)
 *   record events    (scene, group, guid, rec, ...): per record its row events (AddRow / Remove /
 *                    ClearRecord, in call order) then its cell Updates in (row, col) order;
 *                    rrc = op<<24 | rec<<16 | row<<8 | col, op 0 = Update (RECORD_EVENT_DATA::Update,
 *                    old / new the cell), 1 = Add, 2 = Del, 3 = Cover (row events: col 0, old = new = 0).
 *                    In the raw tiles (nfk_outputs) the word also carries the event's slot: bits
 *                    26-31 = slot - tile * rtile_slots (the record tile the event sits in), op in
 *                    bits 24-25; re_slot is NULL.  The nfk_read_* arrays carry the word above.
 *   fired heartbeats (scene, group, guid, kind)
 * Fan-out (GetBroadCastObject recipients): the messages of tile t (property tiles, then record
 * tiles) are one run of msg_cnt[t] recipients at msg_rcpt[msg_base[t]], in event order.  Runs
 * follow each other in tile order; when the frame's k_tick fanned out its own tiles, property
 * tile runs start at a fixed stride (msg_base[t] = t x an upper bound of a tile's messages) and
 * the record tiles' runs follow, densely or (when k_records fanned them out too) at a fixed
 * stride of their own.  Always walk tiles by msg_base / msg_cnt.  ev_moff / re_moff hold the index in msg_rcpt of the
 * event's first recipient; its recipients end where the next event of its tile begins
 * (msg_base[t] + msg_cnt[t] after the tile's last).  When k_tick fanned the property tiles out
 * (fixed-stride runs) ev_moff is NULL, and when k_records fanned the record tiles out re_moff is
 * NULL: such a tile's run holds its events' recipients in event order, the count of each the
 * recipient count of its property's / record's flags for the entity's class (private & !upload: 1,
 * the entity itself; public: the players of its group but itself; else 0).
 * Recipients are slots; slot_obj maps slot -> object index.  nfk_read_fanout returns the dense
 * CSR over [property events ++ record events].
 * nfk_read_* return the same data as dense arrays in object-index terms. */
typedef struct nfk_outputs {
    int32_t n_tiles, tile_slots;     /* property / fired tiles (tile_slots = 256) */
    int32_t n_rtiles, rtile_slots;   /* record-event tiles (rtile_slots = 64) */
    int64_t ev_tile_cap, fi_tile_cap, re_tile_cap;
    const uint32_t* ev_base;   /* [n_tiles + 1]  exclusive scan of per-tile event counts */
    const uint32_t* fi_base;   /* [n_tiles + 1] */
    const uint32_t* re_base;   /* [n_rtiles + 1] */
    const uint32_t* msg_base;  /* [n_tiles + n_rtiles + 1] first message of each tile */
    const uint32_t* msg_cnt;   /* [n_tiles + n_rtiles] messages of each tile */
    const uint32_t* ev_slot; const uint32_t* ev_pid; const uint64_t* ev_old; const uint64_t* ev_new;
    const uint32_t* ev_moff;
    const uint32_t* re_slot; /* NULL: a record event's slot is in its re_rrc word (above) */
    const uint32_t* re_rrc; const uint64_t* re_old; const uint64_t* re_new;
    const uint32_t* re_moff;
    const uint32_t* fi_slot; const uint32_t* fi_kind; const int32_t* fi_remain;
    const uint32_t* msg_rcpt; /* one run per tile (see above) */
    const int32_t* slot_obj;  /* slot -> object index */
    /* object-property events (ev_pid >= n_int + n_flt): ev_old / ev_new hold the NFGUID's data
     * half (nData64), these its head half (nHead64); other events leave them unwritten.  NULL in a
     * world without object properties. */
    const uint64_t* ev_old_h; const uint64_t* ev_new_h;
} nfk_outputs;

/* ---- lifetime: NFCKernelModule ctor/Init/AfterInit (KM:17,51,1490) ---- */
int nfk_create(const nfk_config* cfg, void** out_world);
int nfk_destroy(void* world);
/* human-readable description of the last error on this thread */
const char* nfk_last_error(void);

/* ---- schema: NFIClassModule property/record definitions (KM:137-189) ---- */
int nfk_set_prop_flags(void* world, int32_t cls, const uint8_t* flags /* [n_int+n_flt] */);
int nfk_define_record(void* world, int32_t rec, int32_t rows, int32_t cols,
                      const uint8_t* col_types /* [cols] 0=int64 1=f64 */,
                      const uint8_t* flags_per_class /* [n_class] */);
/* heartbeat kind program; replaces the functor passed to AddSchedule (SM:218) */
int nfk_define_kind(void* world, int32_t kind, const nfk_op* ops, int32_t n_ops);

/* ---- objects: NFCKernelModule::CreateObject (KM:101) ---- */
int nfk_create_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                       const int32_t* scene, const int32_t* group, const uint8_t* cls,
                       const uint8_t* is_player);
/* creation-time property values (CreateObject's config SetProperty, KM:193-208), creation order */
int nfk_load_prop(void* world, int32_t pid, const uint64_t* bits /* [n_objects] */);
/* creation-time object property values (NFGUID head / data halves), creation order */
int nfk_load_object(void* world, int32_t pid, const int64_t* head /* [n_objects] */, const int64_t* data);
/* creation-time record contents, cells [n_objects][cols][rows] as bit patterns, used-row masks */
int nfk_load_record(void* world, int32_t rec, const uint64_t* cells, const uint64_t* used_mask);
/* build the device layout: slots sorted by (scene, group, guid) (NFCSceneInfo group maps) */
int nfk_commit(void* world);

/* ---- runtime membership (after nfk_commit) ----
 * Queued like every other between-frame call and applied at the start of the next nfk_execute,
 * before the queued SetProperty calls, so an entity's events of that frame come from its new
 * scene group.  Slots stay sorted by (scene, group, guid); only the scene groups that changed
 * are rewritten. */
/* property ids SwitchScene writes: SceneID, GroupID (int), X, Y, Z (float); -1 = not in schema */
int nfk_set_scene_props(void* world, int32_t pid_scene, int32_t pid_group, int32_t pid_x, int32_t pid_y,
                        int32_t pid_z);
/* NFCKernelModule::SwitchScene (KM:901-951): leave the group, [GroupID = 0, SceneID = scene when
 * the scene changes], X/Y/Z = (double)x/y/z, GroupID = group, join the new group */
int nfk_switch_scene(void* world, int64_t guid_head, int64_t guid_data, int32_t scene, int32_t group, float x,
                     float y, float z);
/* NFCKernelModule::DestroyObject (KM:273-308): leaves its group, its schedules go with it */
int nfk_destroy_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data);
/* objects ever created in this world (creation-order indices of the nfk_read_* arrays) */
int nfk_object_count(void* world, int32_t* n);
/* An entity's state as a ROW of 64-bit words: properties (prop id order; an object property is two
 * words, data then head), per heartbeat kind its
 * schedule (next, remain|state, start, all|interval), per record its cells [cols][places] and its
 * used-row mask.  A column's cells are in the device's PACKED order, not row order: the used rows
 * first in row order, then the unused rows in row order (a stable partition by the used mask, so the
 * mask alone maps a row to its place and back: place = popcount(used & ((1 << row) - 1)) for a used
 * row, popcount(used) + popcount(~used & ((1 << row) - 1)) for an unused one).  nfk_import_objects
 * takes rows in the same form; a producer or consumer outside export / import must (un)pack by the
 * row's mask.  Rows let a scene shard hand entities to another (SwitchScene across GPUs). */
int nfk_row_words(void* world, int32_t* words);
/* source side: write the entities' rows to rows_dev (device memory, [n][row_words]) on the world's
 * stream, and remove the entities from this world (they must not have other membership calls
 * queued in this window) */
int nfk_export_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                       uint64_t* rows_dev);
/* destination side: new entities with the given rows (device memory, copied on the world's
 * stream before the call returns); also CreateObject after commit (KM:101) */
int nfk_import_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                       const int32_t* scene, const int32_t* group, const uint8_t* cls, const uint8_t* is_player,
                       const uint64_t* rows_dev);
/* CreateObject after commit with creation-time property values from host memory
 * (props [n][n_int + n_flt + 2 n_obj] words: int / f64 bit patterns, then each object property's
 * data and head halves; no schedules, empty records) */
int nfk_spawn_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                      const int32_t* scene, const int32_t* group, const uint8_t* cls, const uint8_t* is_player,
                      const uint64_t* props);

/* ---- property mutation: NFIKernelModule::SetPropertyInt/Float (KM:323,336) ----
 * Queued in call order, applied at the start of the next nfk_execute with the
 * reference's change predicates.  bits = int64 or f64 bit pattern. */
int nfk_set_props(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                  const int32_t* pid, const uint64_t* bits);
/* the same with the objects as nfk's object indices (creation order in this world: the ev_obj /
 * fi_obj of the outputs) for a caller that already resolved the NFGUID (the C++ plugin checks the
 * object exists, KM:325, before it queues): no lookup here; NFK_ERR_NOTFOUND for an index that is
 * not a live object */
int nfk_set_props_obj(void* world, int32_t n, const int32_t* obj, const int32_t* pid, const uint64_t* bits);

/* ---- object properties: NFIKernelModule::SetPropertyObject (KM:362) -> NFCProperty::SetObject
 * (PR:377-416): queued in call order with the other Sets, applied at the start of the next
 * nfk_execute; a value equal to the current NFGUID (both halves) changes nothing and raises no
 * event.  pid must be an object property. */
int nfk_set_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* pid,
                    const int64_t* val_head, const int64_t* val_data);
/* NFIKernelModule::GetPropertyObject (KM:440): read-your-writes like nfk_get_props */
int nfk_get_objects(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* pid,
                    int64_t* val_head, int64_t* val_data);

/* ---- record mutation: NFIKernelModule::SetRecordInt/Float (KM:505, KM:545) ----
 * Queued in call order, applied at the start of the next nfk_execute through NFCRecord::SetInt /
 * SetFloat (RC:182 / RC:243): refused on a row the record does not use (RC:194); an int cell
 * changes when the value differs, an f64 cell unless |new - cur| < 0.001 (TData::operator==).
 * The cell's event of the frame runs from its value before the window's Sets to its value after
 * the frame's record programs (coalesced, dropped when the bits are equal), in (rec, row, col)
 * order beside the programs' events.  is_float (nullable: typed by the column) marks
 * SetRecordFloat calls; a call of the other type than its column writes nothing (RC:189 /
 * RC:250).  NFK_ERR_NOTFOUND for an unknown GUID, NFK_ERR_ARG for a cell outside the record. */
int nfk_set_records(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* rec,
                    const int32_t* row, const int32_t* col, const uint8_t* is_float, const uint64_t* bits);

/* ---- record row operations, queued in call order with the SetRecord calls:
 *   op 1  NFCRecord::AddRow(row, values) (RC:111-180): row -1 = the first unused row (none: nothing
 *         happens); a used row is covered (Cover event, else Add); values [n][NFK_MAX_REC_COLS] words
 *         (NULL or a call without values: the record's initial values, 0), written without Update events
 *   op 2  NFCRecord::Remove(row) (RC:1086-1107): a used row's Del event, then the row is unused (its
 *         cells keep their values)
 *   op 3  NFIKernelModule::ClearRecord (KM:492) -> NFCRecord::Clear (RC:1109): Remove of every row,
 *         the last row first
 * A Set on a row is accepted or refused by the row's used state at that call (RC:194).  The row
 * events are delivered with the frame's record events (rrc op bits, see nfk_outputs).
 * NFK_ERR_NOTFOUND for an unknown GUID, NFK_ERR_ARG for a row outside the record. */
int nfk_record_rows(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* rec,
                    const int32_t* op, const int32_t* row, const uint64_t* values);

/* NFCRecord::IsUsed (RC:1209) for n (object, record) pairs: the used-row masks as the reference holds
 * them now — the device's after the last frame (one read per pair per window, cached until the next
 * nfk_execute) with this window's queued row operations replayed in call order.  What AddRow(-1)
 * would take is the lowest clear bit below the record's rows. */
int nfk_get_used_rows(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* rec,
                      uint64_t* masks);

/* ---- record reads: NFIKernelModule::GetRecordInt/Float (NFIKernelModule.h:134-135) ----
 * NFCRecord::GetInt / GetFloat (RC:616): the cell after the last frame (waits for the world's
 * stream; the used-row masks and cells of all queries in one gather) with this window's queued
 * SetRecord* and row operations on the record replayed in call order (read-your-writes); 0 for a
 * row the record does not use.  NFK_ERR_NOTFOUND / NFK_ERR_ARG as nfk_set_records. */
int nfk_get_records(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* rec,
                    const int32_t* row, const int32_t* col, uint64_t* bits);

/* ---- property reads: NFIKernelModule::GetPropertyInt/Float (KM:401-425) ----
 * The value the reference would return now: the world's value after the last frame (waits for
 * the world's stream) with this window's queued SetProperty* / SwitchScene writes to that
 * property applied on top in call order through the change predicates (read-your-writes).  One
 * 8-byte device read per (entity, property) not read since the last nfk_execute; n > 8 reads are
 * gathered by one kernel.  NFK_ERR_NOTFOUND for an unknown GUID ("There is no object", KM:411). */
int nfk_get_props(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* pid,
                  uint64_t* bits);

/* ---- heartbeats: NFIScheduleModule (SM:218,240,245,251) ---- */
int nfk_add_schedules(void* world, int32_t n, const int64_t* guid_head, const int64_t* guid_data,
                      const int32_t* kind, const float* interval_s, const int32_t* count,
                      const int64_t* now_ms);
/* kind -1: RemoveSchedule(self, name) of a name that has no device program — it removes nothing
 * but still takes the object's remove-list key for this frame (SM:245-249) */
int nfk_remove_schedule(void* world, int64_t guid_head, int64_t guid_data, int32_t kind);
int nfk_remove_all_schedules(void* world, int64_t guid_head, int64_t guid_data);
/* the three calls above batched, in call order: op 1 = AddSchedule(self, kind, interval_s, count)
 * made at now_ms, 2 = RemoveSchedule(self, kind), 3 = RemoveSchedule(self); every GUID and kind is
 * checked before any call is queued */
int nfk_schedule_calls(void* world, int32_t n, const int32_t* op, const int64_t* guid_head, const int64_t* guid_data,
                       const int32_t* kind, const float* interval_s, const int32_t* count, const int64_t* now_ms);
/* the same by object index (see nfk_set_props_obj) */
int nfk_schedule_calls_obj(void* world, int32_t n, const int32_t* op, const int32_t* obj, const int32_t* kind,
                           const float* interval_s, const int32_t* count, const int64_t* now_ms);
/* NFIScheduleModule::ExistSchedule(self, name) (SM:276-285): the object's schedule map as the
 * reference holds it between frames — schedules present after the last frame, minus a
 * RemoveSchedule(self) queued in this window (it erases at once, SM:240); AddSchedule and
 * RemoveSchedule(self, name) take effect in the next Execute.  An unknown GUID reads 0. */
int nfk_exist_schedule(void* world, int64_t guid_head, int64_t guid_data, int32_t kind, int32_t* exists);
/* the AddSchedule calls of the last frame that created a schedule — the (object, name) had none
 * after the frame's removals, so the call's functor is the one that fires from now on (SM:108-116);
 * at most cap entries, *n = how many there are */
int nfk_read_added(void* world, int32_t cap, int32_t* n, int64_t* guid_head, int64_t* guid_data, int32_t* kind);

/* ---- per-Set chains: NFCProperty::SetInt / SetFloat fire a property's per-object callbacks
 * (NFIKernelModule::AddPropertyCallBack, NFIKernelModule.h:40) once per accepted Set (PR:254-334),
 * in the order NFCScheduleModule::Execute runs the heartbeat functors (SM:52-80).  The frame's
 * events are coalesced per (entity, property); for the int / f64 properties named here each
 * nfk_execute also logs every Set its heartbeat programs make that the change predicates accept:
 * (object, kind, op index in the kind's program, property, old, new), so a host with per-object
 * callbacks fires one per Set.  The last Set of an (entity, property) ends at the frame event's new
 * value.  n = 0 watches nothing (no extra kernel runs). */
int nfk_watch_props(void* world, int32_t n, const int32_t* pid);
/* the last nfk_execute's log in the walk's order: objects in NFGUID order, then kind (name order),
 * then op (SM:52-80) — sorted on the device; at most cap entries copied, *n = how many there are
 * (nfk_execute_calls fires nothing and keeps it) */
int nfk_read_chain(void* world, int32_t cap, int32_t* n, int32_t* obj, int32_t* kind, int32_t* op, int32_t* pid,
                   uint64_t* old_bits, uint64_t* new_bits);

/* ---- one server frame: NFCScheduleModule::Execute (SM:49) + NFCKernelModule::Execute (KM:70)
 * + NFCSceneAOIModule::OnPropertyCommonEvent/GetBroadCastObject fan-out (AOI:227,260,531).
 * Asynchronous on the world's stream. */
int nfk_execute(void* world, int64_t now_ms);
/* The calls heartbeat functors made during a frame, applied within that frame: the queued
 * SetProperty / SwitchScene / Create / Destroy / AddSchedule / RemoveSchedule calls take effect
 * and their events and recipient lists replace the outputs, with no heartbeat scan (nothing is
 * due).  In NFCScheduleModule::Execute a functor's Sets land at once (SM:65) and its
 * Add/RemoveSchedule calls are applied at the end of the same walk (SM:83-119); the plugin calls
 * this after running the frame's functors.  Asynchronous like nfk_execute. */
int nfk_execute_calls(void* world);
/* wait for everything queued on the world's stream */
int nfk_sync(void* world);
/* the hipStream_t the world launches on (nfk_config.stream, or the library's own): a caller that
 * moves the world's rows (the scene shards' RCCL transport) orders its work on it */
int nfk_get_stream(void* world, void** stream);
/* synchronise and read the counters of the last tick */
int nfk_summary_get(void* world, nfk_summary* out);
int nfk_outputs_get(void* world, nfk_outputs* out);

/* ---- host copies (synchronising) ---- */
int nfk_read_prop(void* world, int32_t pid, uint64_t* bits /* [n_objects], creation order */);
/* an object property's values, creation order */
int nfk_read_object(void* world, int32_t pid, int64_t* head /* [n_objects] */, int64_t* data);
int nfk_read_record(void* world, int32_t rec, uint64_t* cells /* [n_objects][cols][rows] */);
/* schedule table in creation order: arrays [n_kind][n_objects] */
int nfk_read_schedules(void* world, int64_t* next_ms, int32_t* remain, uint8_t* state);
int nfk_read_events(void* world, int32_t* ev_obj, int32_t* ev_pid, uint64_t* ev_old, uint64_t* ev_new);
/* the head halves of the object-property events, dense like nfk_read_events (0 for other events) */
int nfk_read_events_obj(void* world, uint64_t* ev_old_h, uint64_t* ev_new_h);
int nfk_read_rec_events(void* world, int32_t* re_obj, uint32_t* re_rrc, uint64_t* re_old, uint64_t* re_new);
int nfk_read_fired(void* world, int32_t* fi_obj, int32_t* fi_kind, int32_t* fi_remain);
/* dense CSR over [prop events ++ record events]: msg_off[n_ev + n_re + 1], recipients as objects */
int nfk_read_fanout(void* world, uint32_t* msg_off, int32_t* msg_rcpt_obj);

/* ---- the frame's outputs for a host consumer in ONE read-back ----
 * The host plugin's delivery path (heartbeat functors, common property / record callbacks, AOI
 * recipient lists): the selected outputs of the last frame are compacted on the device into dense
 * arrays in object-index terms (slot -> object, message offsets rebased to a dense CSR over
 * [property events ++ record events]), the fired list optionally ordered by (NFGUID, kind) — the
 * order NFCScheduleModule::Execute walks mObjectScheduleMap (SM:52-80) — with a device radix sort,
 * and copied with one asynchronous copy into a pinned host buffer owned by the world.  The
 * pointers stay valid until the next nfk_execute / nfk_execute_calls / nfk_read_frame.  Arrays not
 * selected are NULL; ev_old_h / ev_new_h are NULL in a world without object properties (0 for
 * the other events). */
#define NFK_READ_FIRED 1u
#define NFK_READ_FIRED_GUID_ORDER 2u /* with NFK_READ_FIRED: (NFGUID, kind) order; else frame order */
#define NFK_READ_EVENTS 4u           /* property and record events */
#define NFK_READ_FANOUT 8u           /* with NFK_READ_EVENTS: the recipient CSR */
typedef struct nfk_frame_host {
    int64_t n_ev, n_re, n_fi, n_msgs;
    const int32_t* ev_obj; const int32_t* ev_pid; const uint64_t* ev_old; const uint64_t* ev_new;
    const uint64_t* ev_old_h; const uint64_t* ev_new_h;
    const int32_t* re_obj; const uint32_t* re_rrc; const uint64_t* re_old; const uint64_t* re_new;
    const int32_t* fi_obj; const int32_t* fi_kind; const int32_t* fi_remain;
    const uint32_t* msg_off;   /* [n_ev + n_re + 1] */
    const int32_t* msg_rcpt;   /* [n_msgs] object indices */
    int64_t bytes;             /* bytes copied to the host */
} nfk_frame_host;
int nfk_read_frame(void* world, uint32_t what, nfk_frame_host* out);

/* ---- leaderboards: NFIRankRedisModule::GetRange (NFCRankRedisModule.cpp:109, a Redis
 * ZREVRANGE 0..k-1 WITH SCORES) with the property as the rank value (SetRankValue takes a double):
 * the k entities of this world with the highest score, ties by NFGUID::ToString() descending
 * (Redis orders equal scores by member, reversed).  Across scene shards, every rank's top k is
 * gathered and merged with the same order (noahgameframe_amd/shard.py rank_top_global). */
int nfk_rank_top(void* world, int32_t pid, int32_t k, int32_t* n_out, int64_t* guid_head, int64_t* guid_data,
                 double* score);

/* ---- schema specialisation ----
 * At nfk_commit k_tick is compiled for the world's schema (its heartbeat programs as straight-line
 * code, its working set and event tables as constants) with hipRTC for gfx950, from the same
 * device source as the library's generic k_tick; the results are bit-identical.  NFGPU_JIT=0 (or
 * a failed compile) keeps the generic kernel. */
/* whether this world's frames run the specialised k_tick; msg: its kernel name or why not */
int nfk_jit_status(void* world, int32_t* on, char* msg, int32_t cap);
/* the specialisation for a schema without a world or a GPU: the generated policy source, and with
 * compile != 0 the hipRTC build for gfx950 (*ok = 1 on success, msg = the compiler log) */
int nfk_jit_preview(int32_t n_int, int32_t n_flt, int32_t n_class, int32_t n_kind,
                    const uint8_t* prop_flags /* [n_class][n_int + n_flt] */,
                    const nfk_op* ops /* [n_kind][NFK_MAX_OPS] */, const int32_t* n_ops /* [n_kind] */,
                    int32_t compile, int32_t* ok, char* src, int32_t src_cap, char* msg, int32_t msg_cap);

/* ---- measurement ---- */
int nfk_set_profiling(void* world, int32_t on);
/* accumulated device time (ms), launch count and algorithmic bytes per kernel:
 * 0 k_tick, 1 k_records, 2 k_fanout, 3 aux (queued host calls), 4 k_scan_tiles,
 * 5 membership changes (k_seg_lists / k_pack / k_unpack / k_meta), 6 k_chain (the per-Set log of
 * the watched properties, nfk_watch_props) */
#define NFK_N_KERNEL_TIMERS 7
int nfk_kernel_times(void* world, double* ms /* [7] */, int64_t* launches /* [7] */, int64_t* bytes /* [7] */);
/* membership changes applied so far: windows that rewrote only the changed scene-group segments
 * (n_seg) or rebuilt the segment table (n_full: a new scene group, or a segment out of slack), and
 * the host milliseconds nfk_execute spent planning them (the device part is timer 5 above) */
int nfk_membership_stats(void* world, int64_t* n_full, int64_t* n_seg, double* host_ms_full, double* host_ms_seg);
int nfk_reset_kernel_times(void* world);

#ifdef __cplusplus
}
#endif
#endif
