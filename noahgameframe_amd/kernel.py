"""Python host mirror of the reference plugin API over the C-ABI (include/nfgpu.h).

`NFKernelModule` keeps the names, argument meaning and failure behaviour of the
reference's NFIKernelModule / NFIScheduleModule calls on the tick path
(NFComm/NFPluginModule/NFIKernelModule.h, NFIScheduleModule.h):
CreateObject, SetPropertyInt/Float, GetPropertyInt/Float, AddSchedule,
RemoveSchedule, Execute.  The compute runs in libnfgpu.so (hand-written HIP
for gfx950).  There is no CPU fallback: constructing a module without the
library or without a GPU raises.
"""
import ctypes
import os

import numpy as np

from . import workload as wl

NFK_MAX_OPS = 8  # include/nfgpu.h: ops per heartbeat program

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NFGPU_LIB") or os.path.join(_HERE, "libnfgpu.so")  # (NFGPU_LIB: A/B timing of library builds)

NFK_OK = 0
_ERRS = {-1: "NFK_ERR_ARG", -2: "NFK_ERR_HIP", -3: "NFK_ERR_STATE", -4: "NFK_ERR_CAPACITY",
         -5: "NFK_ERR_TOUCH", -6: "NFK_ERR_DEVICE", -7: "NFK_ERR_NOTFOUND"}


class NFKError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRS.get(code, code)}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_int32), ("n_int", ctypes.c_int32), ("n_flt", ctypes.c_int32),
                ("n_class", ctypes.c_int32), ("n_kind", ctypes.c_int32), ("n_rec", ctypes.c_int32),
                ("msg_capacity", ctypes.c_int64), ("stream", ctypes.c_void_p), ("slack_per_256", ctypes.c_int32),
                ("n_obj", ctypes.c_int32)]


class Summary(ctypes.Structure):
    _fields_ = [("n_entities", ctypes.c_int64), ("n_prop_events", ctypes.c_int64),
                ("n_rec_events", ctypes.c_int64), ("n_fired", ctypes.c_int64), ("n_msgs", ctypes.c_int64),
                ("alg_bytes_tick", ctypes.c_int64), ("alg_bytes_rec", ctypes.c_int64),
                ("alg_bytes_fan", ctypes.c_int64), ("device_error", ctypes.c_int32), ("tick", ctypes.c_int32)]


class Outputs(ctypes.Structure):
    """nfk_outputs: tile-staged device outputs of the last frame (see include/nfgpu.h)."""
    _fields_ = ([("n_tiles", ctypes.c_int32), ("tile_slots", ctypes.c_int32), ("n_rtiles", ctypes.c_int32),
                 ("rtile_slots", ctypes.c_int32), ("ev_tile_cap", ctypes.c_int64), ("fi_tile_cap", ctypes.c_int64),
                 ("re_tile_cap", ctypes.c_int64)] +
                [(n, ctypes.c_void_p) for n in
                 ["ev_base", "fi_base", "re_base", "msg_base", "msg_cnt", "ev_slot", "ev_pid", "ev_old", "ev_new", "ev_moff",
                  "re_slot", "re_rrc", "re_old", "re_new", "re_moff", "fi_slot", "fi_kind", "fi_remain",
                  "msg_rcpt", "slot_obj", "ev_old_h", "ev_new_h"]])


N_KERNEL_TIMERS = 7
KERNEL_TIMER_NAMES = ["k_tick", "k_records", "k_fanout", "aux", "k_scan_tiles", "membership", "k_chain"]


_lib = None


def load_library(path=LIB_PATH):
    """Load libnfgpu.so; raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(path)
    P, I32, I64, VP = ctypes.POINTER, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
    sig = {
        "nfk_create": [P(Config), P(VP)], "nfk_destroy": [VP], "nfk_last_error": [],
        "nfk_set_prop_flags": [VP, I32, VP], "nfk_define_record": [VP, I32, I32, I32, VP, VP],
        "nfk_define_kind": [VP, I32, VP, I32],
        "nfk_create_objects": [VP, I32, VP, VP, VP, VP, VP, VP], "nfk_load_prop": [VP, I32, VP],
        "nfk_load_record": [VP, I32, VP, VP], "nfk_commit": [VP],
        "nfk_set_props": [VP, I32, VP, VP, VP, VP], "nfk_set_props_obj": [VP, I32, VP, VP, VP], "nfk_set_records": [VP, I32, VP, VP, VP, VP, VP, VP, VP],
        "nfk_get_records": [VP, I32, VP, VP, VP, VP, VP, VP],
        "nfk_add_schedules": [VP, I32, VP, VP, VP, VP, VP, VP],
        "nfk_remove_schedule": [VP, I64, I64, I32], "nfk_remove_all_schedules": [VP, I64, I64],
        "nfk_schedule_calls": [VP, I32, VP, VP, VP, VP, VP, VP, VP], "nfk_schedule_calls_obj": [VP, I32, VP, VP, VP, VP, VP, VP],
        "nfk_get_props": [VP, I32, VP, VP, VP, VP], "nfk_exist_schedule": [VP, I64, I64, I32, VP],
        "nfk_execute": [VP, I64], "nfk_execute_calls": [VP], "nfk_summary_get": [VP, P(Summary)], "nfk_outputs_get": [VP, P(Outputs)],
        "nfk_read_prop": [VP, I32, VP], "nfk_read_record": [VP, I32, VP], "nfk_read_schedules": [VP, VP, VP, VP],
        "nfk_read_events": [VP, VP, VP, VP, VP], "nfk_read_rec_events": [VP, VP, VP, VP, VP],
        "nfk_read_fired": [VP, VP, VP, VP], "nfk_read_fanout": [VP, VP, VP],
        "nfk_set_profiling": [VP, I32], "nfk_kernel_times": [VP, VP, VP, VP], "nfk_reset_kernel_times": [VP],
        "nfk_set_scene_props": [VP, I32, I32, I32, I32, I32],
        "nfk_switch_scene": [VP, I64, I64, I32, I32, ctypes.c_float, ctypes.c_float, ctypes.c_float],
        "nfk_destroy_objects": [VP, I32, VP, VP], "nfk_object_count": [VP, VP], "nfk_row_words": [VP, VP],
        "nfk_export_objects": [VP, I32, VP, VP, VP],
        "nfk_import_objects": [VP, I32, VP, VP, VP, VP, VP, VP, VP],
        "nfk_spawn_objects": [VP, I32, VP, VP, VP, VP, VP, VP, VP], "nfk_sync": [VP],
        "nfk_rank_top": [VP, I32, I32, VP, VP, VP, VP],
        "nfk_jit_status": [VP, VP, VP, I32], "nfk_membership_stats": [VP, VP, VP, VP, VP],
        "nfk_jit_preview": [I32, I32, I32, I32, VP, VP, VP, I32, VP, VP, I32, VP, I32],
        "nfk_load_object": [VP, I32, VP, VP], "nfk_set_objects": [VP, I32, VP, VP, VP, VP, VP],
        "nfk_get_objects": [VP, I32, VP, VP, VP, VP, VP], "nfk_read_object": [VP, I32, VP, VP],
        "nfk_read_events_obj": [VP, VP, VP], "nfk_record_rows": [VP, I32, VP, VP, VP, VP, VP, VP],
    }
    for name, args in sig.items():
        if not hasattr(lib, name) and os.environ.get("NFGPU_LIB"):
            continue   # (A/B timing of an older library build: entry points it predates stay unbound)
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_char_p if name == "nfk_last_error" else ctypes.c_int
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class NFKernelModule:
    """One GPU-resident world (the entities of one scene shard)."""

    def __init__(self, capacity, n_int=wl.N_INT, n_flt=wl.N_FLT, n_class=2, n_kind=len(wl.KINDS), n_rec=0,
                 msg_capacity=0, stream=None, slack_per_256=0, n_oprops=0):
        self.lib = load_library()
        cfg = Config(capacity, n_int, n_flt, n_class, n_kind, n_rec, msg_capacity, stream, slack_per_256, n_oprops)
        self.n_oprops = n_oprops
        h = ctypes.c_void_p()
        self._chk(self.lib.nfk_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.stream = stream
        self.n_int, self.n_flt, self.n_kind, self.n_rec = n_int, n_flt, n_kind, n_rec
        self.n_obj = 0
        self.rec_shape = {}

    def _chk(self, rc):
        if rc != NFK_OK:
            raise NFKError(rc, self.lib.nfk_last_error().decode())
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.nfk_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- schema (NFIClassModule) ----
    def set_prop_flags(self, cls, flags):
        flags = np.ascontiguousarray(flags, np.uint8)
        self._chk(self.lib.nfk_set_prop_flags(self.h, cls, _p(flags)))

    def define_record(self, rec, rows, cols, col_types, flags_per_class):
        ct = np.ascontiguousarray(col_types, np.uint8)
        fl = np.ascontiguousarray(flags_per_class, np.uint8)
        self._chk(self.lib.nfk_define_record(self.h, rec, rows, cols, _p(ct), _p(fl)))
        self.rec_shape[rec] = (cols, rows)

    def define_kind(self, kind, ops):
        ops = np.ascontiguousarray(ops)
        if ops.dtype != wl.OP_DTYPE:
            ops = ops.view(wl.OP_DTYPE).reshape(-1)
        self._chk(self.lib.nfk_define_kind(self.h, kind, _p(ops), len(ops)))

    # ---- objects (NFIKernelModule::CreateObject) ----
    def create_objects(self, guid_head, guid_data, scene, group, cls, is_player):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (scene, np.int32), (group, np.int32),
              (cls, np.uint8), (is_player, np.uint8))]
        self._chk(self.lib.nfk_create_objects(self.h, len(a[0]), *[_p(x) for x in a]))
        self._keep = getattr(self, "_keep", []) + [a]
        self.n_obj += len(a[0])

    def load_prop(self, pid, values):
        v = np.ascontiguousarray(values)
        bits = v.view(np.uint64) if v.dtype.itemsize == 8 else v.astype(np.int64).view(np.uint64)
        self._chk(self.lib.nfk_load_prop(self.h, pid, _p(np.ascontiguousarray(bits))))

    def load_object(self, pid, head, data):
        h = np.ascontiguousarray(head, np.int64)
        d = np.ascontiguousarray(data, np.int64)
        self._chk(self.lib.nfk_load_object(self.h, pid, _p(h), _p(d)))

    def load_record(self, rec, cells, used):
        c = np.ascontiguousarray(cells, np.uint64)
        u = np.ascontiguousarray(used, np.uint64)
        self._chk(self.lib.nfk_load_record(self.h, rec, _p(c), _p(u)))

    def commit(self):
        self._chk(self.lib.nfk_commit(self.h))

    # ---- NFIKernelModule::SetProperty* (queued, applied at the next Execute) ----
    def set_props(self, guid_head, guid_data, pid, bits):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (pid, np.int32), (bits, np.uint64))]
        self._chk(self.lib.nfk_set_props(self.h, len(a[0]), *[_p(x) for x in a]))

    def set_props_obj(self, obj, pid, bits):
        """nfk_set_props_obj: the same calls by nfk object index (creation order; the outputs' ev_obj)."""
        a = [np.ascontiguousarray(x, t) for x, t in ((obj, np.int32), (pid, np.int32), (bits, np.uint64))]
        self._chk(self.lib.nfk_set_props_obj(self.h, len(a[0]), *[_p(x) for x in a]))

    # ---- NFIKernelModule::SetPropertyObject / GetPropertyObject (KM:362 / KM:440) ----
    def set_objects(self, guid_head, guid_data, pid, val_head, val_data):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (pid, np.int32), (val_head, np.int64),
              (val_data, np.int64))]
        self._chk(self.lib.nfk_set_objects(self.h, len(a[0]), *[_p(x) for x in a]))

    def get_objects(self, guid_head, guid_data, pid):
        a = [np.ascontiguousarray(x, t) for x, t in ((guid_head, np.int64), (guid_data, np.int64), (pid, np.int32))]
        vh = np.zeros(len(a[0]), np.int64)
        vd = np.zeros(len(a[0]), np.int64)
        self._chk(self.lib.nfk_get_objects(self.h, len(a[0]), *[_p(x) for x in a], _p(vh), _p(vd)))
        return vh, vd

    def SetPropertyObject(self, guid, pid, value):
        self.set_objects([guid[0]], [guid[1]], [pid], [value[0]], [value[1]])
        return True

    def GetPropertyObject(self, guid, pid):
        vh, vd = self.get_objects([guid[0]], [guid[1]], [pid])
        return int(vh[0]), int(vd[0])

    def read_object(self, pid):
        h = np.zeros(self.n_obj, np.int64)
        d = np.zeros(self.n_obj, np.int64)
        self._chk(self.lib.nfk_read_object(self.h, pid, _p(h), _p(d)))
        return h, d

    # ---- NFIKernelModule::SetRecordInt / SetRecordFloat ----
    def set_records(self, guid_head, guid_data, rec, row, col, bits, is_float=None):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (rec, np.int32), (row, np.int32), (col, np.int32))]
        f = None if is_float is None else np.ascontiguousarray(is_float, np.uint8)
        b = np.ascontiguousarray(bits, np.uint64)
        self._chk(self.lib.nfk_set_records(self.h, len(a[0]), *[_p(x) for x in a], _p(f) if f is not None else None,
                                           _p(b)))

    def record_rows(self, guid_head, guid_data, rec, op, row, values=None):
        """NFCRecord::AddRow (op 1, row -1 = first unused, values [n][16] words) / Remove (op 2) /
        NFIKernelModule::ClearRecord (op 3), queued in call order with the SetRecord calls"""
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (rec, np.int32), (op, np.int32), (row, np.int32))]
        v = None if values is None else np.ascontiguousarray(values, np.uint64).reshape(len(a[0]), 16)
        self._chk(self.lib.nfk_record_rows(self.h, len(a[0]), *[_p(x) for x in a], _p(v)))

    def AddRow(self, guid, rec, row=-1, values=None):
        self.record_rows([guid[0]], [guid[1]], [rec], [1], [row], None if values is None else [values])
        return True

    def RemoveRow(self, guid, rec, row):
        self.record_rows([guid[0]], [guid[1]], [rec], [2], [row])
        return True

    def ClearRecord(self, guid, rec):
        self.record_rows([guid[0]], [guid[1]], [rec], [3], [0])
        return True

    def get_records(self, guid_head, guid_data, rec, row, col):
        """NFIKernelModule::GetRecordInt/Float for n cells: raw 64-bit patterns, read-your-writes"""
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (rec, np.int32), (row, np.int32), (col, np.int32))]
        out = np.zeros(len(a[0]), np.uint64)
        self._chk(self.lib.nfk_get_records(self.h, len(a[0]), *[_p(x) for x in a], _p(out)))
        return out

    def SetRecordInt(self, guid, rec, row, col, value):
        self.set_records([guid[0]], [guid[1]], [rec], [row], [col], [np.int64(value).view(np.uint64)], [0])
        return True

    def SetRecordFloat(self, guid, rec, row, col, value):
        self.set_records([guid[0]], [guid[1]], [rec], [row], [col], [np.float64(value).view(np.uint64)], [1])
        return True

    def SetPropertyInt(self, guid, prop, value):
        pid = wl.PID[prop] if isinstance(prop, str) else prop
        self.set_props([guid[0]], [guid[1]], [pid], [np.int64(value).view(np.uint64)])
        return True

    def SetPropertyFloat(self, guid, prop, value):
        pid = wl.PID[prop] if isinstance(prop, str) else prop
        self.set_props([guid[0]], [guid[1]], [pid], [np.float64(value).view(np.uint64)])
        return True

    # ---- NFIScheduleModule ----
    def add_schedules(self, guid_head, guid_data, kind, interval_s, count, now_ms):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (kind, np.int32), (interval_s, np.float32),
              (count, np.int32), (now_ms, np.int64))]
        self._chk(self.lib.nfk_add_schedules(self.h, len(a[0]), *[_p(x) for x in a]))

    def AddSchedule(self, guid, name, interval_s, count, now_ms):
        kind = wl.KID[name] if isinstance(name, str) else name
        self.add_schedules([guid[0]], [guid[1]], [kind], [interval_s], [count], [now_ms])
        return True

    def schedule_calls(self, op, guid_head, guid_data, kind, interval_s, count, now_ms):
        """AddSchedule (op 1) / RemoveSchedule(self, name) (op 2) / RemoveSchedule(self) (op 3)
        calls in call order, as one batch."""
        a = [np.ascontiguousarray(x, t) for x, t in
             ((op, np.int32), (guid_head, np.int64), (guid_data, np.int64), (kind, np.int32),
              (interval_s, np.float32), (count, np.int32), (now_ms, np.int64))]
        self._chk(self.lib.nfk_schedule_calls(self.h, len(a[0]), *[_p(x) for x in a]))

    def schedule_calls_obj(self, op, obj, kind, interval_s, count, now_ms):
        """nfk_schedule_calls_obj: schedule_calls by nfk object index."""
        a = [np.ascontiguousarray(x, t) for x, t in
             ((op, np.int32), (obj, np.int32), (kind, np.int32), (interval_s, np.float32), (count, np.int32),
              (now_ms, np.int64))]
        self._chk(self.lib.nfk_schedule_calls_obj(self.h, len(a[0]), *[_p(x) for x in a]))

    def RemoveSchedule(self, guid, name=None):
        if name is None:
            self._chk(self.lib.nfk_remove_all_schedules(self.h, int(guid[0]), int(guid[1])))
        else:
            kind = wl.KID[name] if isinstance(name, str) else name
            self._chk(self.lib.nfk_remove_schedule(self.h, int(guid[0]), int(guid[1]), kind))
        return True

    # ---- runtime membership (NFCKernelModule::SwitchScene / DestroyObject / CreateObject) ----
    def set_scene_props(self, pid_scene, pid_group, pid_x, pid_y, pid_z):
        self._chk(self.lib.nfk_set_scene_props(self.h, pid_scene, pid_group, pid_x, pid_y, pid_z))

    def SwitchScene(self, guid, scene, group, x, y, z):
        self._chk(self.lib.nfk_switch_scene(self.h, int(guid[0]), int(guid[1]), int(scene), int(group),
                                            float(x), float(y), float(z)))
        return True

    def destroy_objects(self, guid_head, guid_data):
        a = [np.ascontiguousarray(x, np.int64) for x in (guid_head, guid_data)]
        self._chk(self.lib.nfk_destroy_objects(self.h, len(a[0]), _p(a[0]), _p(a[1])))

    def DestroyObject(self, guid):
        self.destroy_objects([guid[0]], [guid[1]])
        return True

    def object_count(self):
        n = ctypes.c_int32()
        self._chk(self.lib.nfk_object_count(self.h, ctypes.byref(n)))
        return n.value

    def membership_stats(self):
        """{n_full, n_seg, host_ms_full, host_ms_seg}: membership windows applied by rebuilding the
        segment table / by rewriting only changed segments, and their host planning time"""
        nf, ns = ctypes.c_int64(), ctypes.c_int64()
        mf, ms = ctypes.c_double(), ctypes.c_double()
        self._chk(self.lib.nfk_membership_stats(self.h, ctypes.byref(nf), ctypes.byref(ns), ctypes.byref(mf),
                                                ctypes.byref(ms)))
        return {"n_full": nf.value, "n_seg": ns.value, "host_ms_full": mf.value, "host_ms_seg": ms.value}

    def jit_status(self):
        """(True, message) when k_tick runs the hipRTC specialisation built at commit"""
        on = ctypes.c_int32()
        msg = ctypes.create_string_buffer(4096)
        self._chk(self.lib.nfk_jit_status(self.h, ctypes.byref(on), msg, len(msg)))
        return bool(on.value), msg.value.decode()

    def row_words(self):
        n = ctypes.c_int32()
        self._chk(self.lib.nfk_row_words(self.h, ctypes.byref(n)))
        return n.value

    def export_objects(self, guid_head, guid_data, rows_dev_ptr):
        """Pack the entities' state rows into device memory at rows_dev_ptr ([n][row_words] u64)
        on the world's stream and remove them from this world."""
        a = [np.ascontiguousarray(x, np.int64) for x in (guid_head, guid_data)]
        self._chk(self.lib.nfk_export_objects(self.h, len(a[0]), _p(a[0]), _p(a[1]), ctypes.c_void_p(rows_dev_ptr)))

    def import_objects(self, guid_head, guid_data, scene, group, cls, is_player, rows_dev_ptr):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (scene, np.int32), (group, np.int32),
              (cls, np.uint8), (is_player, np.uint8))]
        self._chk(self.lib.nfk_import_objects(self.h, len(a[0]), *[_p(x) for x in a], ctypes.c_void_p(rows_dev_ptr)))
        self.n_obj = self.object_count()

    def spawn_objects(self, guid_head, guid_data, scene, group, cls, is_player, props):
        a = [np.ascontiguousarray(x, t) for x, t in
             ((guid_head, np.int64), (guid_data, np.int64), (scene, np.int32), (group, np.int32),
              (cls, np.uint8), (is_player, np.uint8))]
        pr = np.ascontiguousarray(props, np.uint64)
        self._chk(self.lib.nfk_spawn_objects(self.h, len(a[0]), *[_p(x) for x in a], _p(pr)))
        self.n_obj = self.object_count()

    # ---- leaderboards (NFIRankRedisModule::GetRange) ----
    def rank_top(self, prop, k):
        """The k entities with the highest score (the property as a double), ties by
        NFGUID::ToString() descending: (guid_head, guid_data, score) arrays."""
        pid = wl.PID[prop] if isinstance(prop, str) else int(prop)
        gh = np.zeros(max(k, 1), np.int64)
        gd = np.zeros(max(k, 1), np.int64)
        sc = np.zeros(max(k, 1), np.float64)
        n = ctypes.c_int32()
        self._chk(self.lib.nfk_rank_top(self.h, pid, int(k), ctypes.byref(n), _p(gh), _p(gd), _p(sc)))
        return gh[:n.value], gd[:n.value], sc[:n.value]

    # ---- one frame ----
    def Execute(self, now_ms):
        self._chk(self.lib.nfk_execute(self.h, int(now_ms)))
        return True

    def ExecuteCalls(self):
        """nfk_execute_calls: the queued calls applied in a pass where nothing fires (what heartbeat
        functors call inside NFCScheduleModule::Execute's walk, SM:65, SM:83-119)."""
        self._chk(self.lib.nfk_execute_calls(self.h))
        return True

    def synchronize(self):
        self._chk(self.lib.nfk_sync(self.h))

    def summary(self):
        s = Summary()
        self._chk(self.lib.nfk_summary_get(self.h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in Summary._fields_}

    def outputs(self):
        o = Outputs()
        self._chk(self.lib.nfk_outputs_get(self.h, ctypes.byref(o)))
        return {f: getattr(o, f) for f, _ in Outputs._fields_}

    def outputs_raw(self):
        """nfk_outputs_get into one reused struct (device pointers; the frame's dense ranks are
        built asynchronously on the world's stream) — what a consumer calls every frame."""
        if not hasattr(self, "_out"):
            self._out = Outputs()
        self._chk(self.lib.nfk_outputs_get(self.h, ctypes.byref(self._out)))
        return self._out

    # ---- readback ----
    def read_prop(self, pid):
        out = np.zeros(self.n_obj, np.uint64)
        self._chk(self.lib.nfk_read_prop(self.h, pid, _p(out)))
        return out.view(np.int64) if pid < self.n_int else out.view(np.float64)

    def get_props(self, guid_head, guid_data, pid):
        """NFIKernelModule::GetProperty* for n (entity, property) pairs: the value after the last
        frame with this window's queued writes applied (read-your-writes); raw 64-bit patterns."""
        a = [np.ascontiguousarray(x, t) for x, t in ((guid_head, np.int64), (guid_data, np.int64), (pid, np.int32))]
        out = np.zeros(len(a[0]), np.uint64)
        self._chk(self.lib.nfk_get_props(self.h, len(a[0]), *[_p(x) for x in a], _p(out)))
        return out

    def GetPropertyInt(self, guid, prop):
        pid = wl.PID[prop] if isinstance(prop, str) else prop
        return int(self.get_props([guid[0]], [guid[1]], [pid]).view(np.int64)[0])

    def GetPropertyFloat(self, guid, prop):
        pid = wl.PID[prop] if isinstance(prop, str) else prop
        return float(self.get_props([guid[0]], [guid[1]], [pid]).view(np.float64)[0])

    def ExistSchedule(self, guid, name):
        kind = wl.KID[name] if isinstance(name, str) else name
        e = ctypes.c_int32()
        self._chk(self.lib.nfk_exist_schedule(self.h, int(guid[0]), int(guid[1]), int(kind), ctypes.byref(e)))
        return bool(e.value)

    def read_record(self, rec):
        cols, rows = self.rec_shape[rec]
        out = np.zeros((self.n_obj, cols, rows), np.uint64)
        self._chk(self.lib.nfk_read_record(self.h, rec, _p(out)))
        return out

    def read_schedules(self):
        nx = np.zeros((self.n_kind, self.n_obj), np.int64)
        rm = np.zeros((self.n_kind, self.n_obj), np.int32)
        st = np.zeros((self.n_kind, self.n_obj), np.uint8)
        self._chk(self.lib.nfk_read_schedules(self.h, _p(nx), _p(rm), _p(st)))
        return nx, rm, st

    def read_tick(self):
        """All outputs of the last frame, entities as object (creation) indices."""
        s = self.summary()
        ne, nr, nf, nm = s["n_prop_events"], s["n_rec_events"], s["n_fired"], s["n_msgs"]
        ev = [np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne, np.uint64), np.zeros(ne, np.uint64)]
        self._chk(self.lib.nfk_read_events(self.h, *[_p(x) for x in ev]))
        re = [np.zeros(nr, np.int32), np.zeros(nr, np.uint32), np.zeros(nr, np.uint64), np.zeros(nr, np.uint64)]
        self._chk(self.lib.nfk_read_rec_events(self.h, *[_p(x) for x in re]))
        fi = [np.zeros(nf, np.int32), np.zeros(nf, np.int32), np.zeros(nf, np.int32)]
        self._chk(self.lib.nfk_read_fired(self.h, *[_p(x) for x in fi]))
        mo = np.zeros(ne + nr + 1, np.uint32)
        mr = np.zeros(nm, np.int32)
        self._chk(self.lib.nfk_read_fanout(self.h, _p(mo), _p(mr)))
        out = dict(ev_obj=ev[0], ev_pid=ev[1], ev_old=ev[2], ev_new=ev[3],
                   re_obj=re[0], re_rrc=re[1], re_old=re[2], re_new=re[3],
                   fi_obj=fi[0], fi_kind=fi[1], fi_rem=fi[2], mo_off=mo, mr_obj=mr, summary=s)
        if self.n_oprops:
            oh = [np.zeros(ne, np.uint64), np.zeros(ne, np.uint64)]
            self._chk(self.lib.nfk_read_events_obj(self.h, *[_p(x) for x in oh]))
            out["ev_oldh"], out["ev_newh"] = oh
        return out

    # ---- measurement ----
    def set_profiling(self, on):
        self._chk(self.lib.nfk_set_profiling(self.h, 1 if on else 0))

    def kernel_times(self):
        ms = np.zeros(N_KERNEL_TIMERS, np.float64)
        n = np.zeros(N_KERNEL_TIMERS, np.int64)
        b = np.zeros(N_KERNEL_TIMERS, np.int64)
        self._chk(self.lib.nfk_kernel_times(self.h, _p(ms), _p(n), _p(b)))
        return ms, n, b

    def reset_kernel_times(self):
        self._chk(self.lib.nfk_reset_kernel_times(self.h))


def jit_preview(w, compile=False):
    """nfk_jit_preview: the k_tick schema policy (JitSchema source) nfk_commit would generate for a
    workload's schema, and with compile=True whether hipRTC builds k_tick<.., JitSchema> for gfx950
    from it.  Needs no GPU.  Returns (source, ok, message)."""
    lib = load_library()
    _, n_int, n_flt, n_cls, n_kind = (int(x) for x in w["cfg"][:5])
    flags = np.ascontiguousarray(np.asarray(w["prop_flags"])[:n_cls], np.uint8)
    src_ops = np.asarray(w["ops"][:n_kind])
    if src_ops.dtype != wl.OP_DTYPE:  # (raw records from a workload file)
        src_ops = src_ops.view(wl.OP_DTYPE).reshape(n_kind, -1)
    ops = np.zeros((n_kind, NFK_MAX_OPS), wl.OP_DTYPE)  # [n_kind][NFK_MAX_OPS] (nfgpu.h)
    ops[:, :src_ops.shape[1]] = src_ops
    n_ops = np.ascontiguousarray(w["n_ops"][:n_kind], np.int32)
    ok = ctypes.c_int32()
    src = ctypes.create_string_buffer(1 << 20)
    msg = ctypes.create_string_buffer(1 << 16)
    rc = lib.nfk_jit_preview(n_int, n_flt, n_cls, n_kind, _p(flags), _p(ops), _p(n_ops), int(compile),
                             ctypes.byref(ok), src, len(src), msg, len(msg))
    if rc != NFK_OK:
        raise NFKError(rc, lib.nfk_last_error().decode())
    return src.value.decode(), bool(ok.value), msg.value.decode()


def world_from_workload(w, capacity=None, msg_capacity=0, stream=None, slack_per_256=0):
    """Build an NFKernelModule from a workload dict (see workload.make_world): classes,
    kinds, objects, creation-time values, then the AddSchedule calls made before frame 0."""
    cfg = w["cfg"]
    n_obj, n_int, n_flt, n_cls, n_kind, n_rec = (int(x) for x in cfg[:6])
    n_op = int(w["n_oprops"][0]) if "n_oprops" in w else 0
    m = NFKernelModule(capacity or n_obj, n_int, n_flt, n_cls, n_kind, n_rec, msg_capacity, stream, slack_per_256,
                       n_op)
    if "scene_props" in w:
        m.set_scene_props(*(int(x) for x in w["scene_props"]))
    m.cur_scene = np.array(w["scene"], np.int32)   # membership as SwitchScene calls change it
    m.cur_group = np.array(w["group"], np.int32)
    for c in range(n_cls):
        m.set_prop_flags(c, w["prop_flags"][c])
    for r in range(n_rec):
        m.define_record(r, int(w["rec_rows"][r]), int(w["rec_cols"][r]), w["rec_ctype"][r],
                        w["rec_flags"][:, r])
    for k in range(n_kind):
        m.define_kind(k, w["ops"][k][: int(w["n_ops"][k])])
    # objects created before frame 0 (a workload's later objects, born[o] >= 0, are the last ones
    # and enter through nfk_spawn_objects in their window: run_workload)
    n0 = int(np.sum(w["born"] < 0)) if "born" in w else n_obj
    m.create_objects(w["guid_head"][:n0], w["guid_data"][:n0], w["scene"][:n0], w["group"][:n0], w["cls"][:n0],
                     w["is_player"][:n0])
    for p in range(n_int):
        m.load_prop(p, w["init_i"][p][:n0])
    for p in range(n_flt):
        m.load_prop(n_int + p, w["init_f"][p][:n0])
    for p in range(n_op):
        m.load_object(n_int + n_flt + p, w["init_oh"][p][:n0], w["init_od"][p][:n0])
    for r in range(n_rec):
        m.load_record(r, w[f"rec{r}_cells"][:n0], w[f"rec{r}_used"][:n0])
    m.commit()
    gh, gd = w["guid_head"], w["guid_data"]
    so = w["s_obj"]
    m.add_schedules(gh[so], gd[so], w["s_kind"], w["s_interval"], w["s_count"], w["s_time"])
    return m


def run_workload(m, w, tick, collect=True):
    """Replay the between-frame calls of frame `tick` in the oracle's window order — CreateObject
    (nfk_spawn_objects), SwitchScene, schedule calls, SetProperty calls, SetRecord calls,
    DestroyObject — then Execute it."""
    gh, gd = w["guid_head"], w["guid_data"]
    if "born" in w:
        new = np.nonzero(w["born"] == tick)[0]
        if len(new):
            parts = [w["init_i"][:, new].astype(np.int64).view(np.uint64),
                     w["init_f"][:, new].astype(np.float64).view(np.uint64)]
            if m.n_oprops:   # each object property as (data, head)
                od = w["init_od"][:, new].astype(np.int64).view(np.uint64)
                oh = w["init_oh"][:, new].astype(np.int64).view(np.uint64)
                parts.append(np.stack([od, oh], 1).reshape(-1, len(new)))
            props = np.concatenate(parts).T
            m.spawn_objects(gh[new], gd[new], w["scene"][new], w["group"][new], w["cls"][new], w["is_player"][new],
                            np.ascontiguousarray(props))
    if "sw_tick" in w:
        for i in np.nonzero(w["sw_tick"] == tick)[0]:
            o = int(w["sw_obj"][i])
            sc, gr = int(w["sw_scene"][i]), int(w["sw_group"][i])
            if sc < 0:   # the object's own cell
                sc, gr = int(m.cur_scene[o]), int(m.cur_group[o])
            m.SwitchScene((int(gh[o]), int(gd[o])), sc, gr, w["sw_x"][i], w["sw_y"][i], w["sw_z"][i])
            m.cur_scene[o], m.cur_group[o] = sc, gr
    # (by_object: the calls by nfk object index — nfk_set_props_obj / nfk_schedule_calls_obj — which
    # in a world without objects created after commit is the workload's object index)
    by_object = os.environ.get("NFGPU_TEST_BY_OBJECT") == "1" and "born" not in w
    hsel = np.nonzero(w["h_tick"] == tick)[0]
    if len(hsel):   # call order preserved
        ho = w["h_obj"][hsel]
        if by_object:
            m.schedule_calls_obj(w["h_op"][hsel], ho, w["h_kind"][hsel], w["h_interval"][hsel], w["h_count"][hsel],
                                 w["h_time"][hsel])
        else:
            m.schedule_calls(w["h_op"][hsel], gh[ho], gd[ho], w["h_kind"][hsel], w["h_interval"][hsel],
                             w["h_count"][hsel], w["h_time"][hsel])
    xsel = np.nonzero(w["x_tick"] == tick)[0]
    if len(xsel):
        mode = w["x_mode"][xsel] if "x_mode" in w else np.zeros(len(xsel), np.uint8)
        # runs of plain SetProperty calls go as one batch; a read-modify-write call (mode 1:
        # SetProperty(p, GetProperty(p) + delta)) reads through nfk_get_props first
        cut = np.nonzero(np.diff(np.concatenate([[2], mode, [2]])))[0]
        for a, b in zip(cut[:-1], cut[1:]):
            sel = xsel[a:b]
            xo = w["x_obj"][sel]
            if mode[a] == 0:
                pid = w["x_pid"][sel]
                isobj = pid >= m.n_int + m.n_flt
                # (calls on different properties never interact: the object calls go as their own batch)
                if (~isobj).any() and by_object:
                    m.set_props_obj(xo[~isobj], pid[~isobj], w["x_bits"][sel][~isobj])
                elif (~isobj).any():
                    m.set_props(gh[xo[~isobj]], gd[xo[~isobj]], pid[~isobj], w["x_bits"][sel][~isobj])
                if isobj.any():
                    m.set_objects(gh[xo[isobj]], gd[xo[isobj]], pid[isobj], w["x_bits_h"][sel][isobj].view(np.int64),
                                  w["x_bits"][sel][isobj].view(np.int64))
                continue
            for i in sel:
                o, p = int(w["x_obj"][i]), int(w["x_pid"][i])
                cur = m.get_props([gh[o]], [gd[o]], [p])
                d = w["x_bits"][i:i + 1]
                if p < m.n_int:
                    v = (cur.view(np.int64) + d.view(np.int64)).view(np.uint64)
                else:
                    v = (cur.view(np.float64) + d.view(np.float64)).view(np.uint64)
                m.set_props([gh[o]], [gd[o]], [p], v)
    if "r_tick" in w:   # SetRecordInt / SetRecordFloat calls (typed by their column), row operations
        rsel = np.nonzero(w["r_tick"] == tick)[0]
        if len(rsel):
            ops = w["r_op"][rsel] if "r_op" in w else np.zeros(len(rsel), np.uint8)
            cut = np.nonzero(np.diff(np.concatenate([[-1], (ops != 0).astype(np.int8), [-1]])))[0]
            for a, b in zip(cut[:-1], cut[1:]):   # runs of Sets / of row operations, in call order
                sel = rsel[a:b]
                ro = w["r_obj"][sel]
                if ops[a] == 0:
                    m.set_records(gh[ro], gd[ro], w["r_rec"][sel], w["r_row"][sel], w["r_col"][sel], w["r_bits"][sel])
                else:
                    m.record_rows(gh[ro], gd[ro], w["r_rec"][sel], ops[a:b].astype(np.int32), w["r_row"][sel],
                                  w["r_vals"][sel])
    if "d_tick" in w:
        dead = w["d_obj"][w["d_tick"] == tick]
        if len(dead):
            m.destroy_objects(gh[dead], gd[dead])
    now = int(w["tick_time"][tick])
    if now == np.iinfo(np.int64).min:  # a calls-only pass (nfk_execute_calls: nothing fires)
        m.ExecuteCalls()
    else:
        m.Execute(now)
    return m.read_tick() if collect else None
