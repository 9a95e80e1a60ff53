"""ctypes signatures of libedl_runtime.so (csrc/runtime)."""
import ctypes

vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_int64
u64 = ctypes.c_uint64
cp = ctypes.c_char_p
u64p = ctypes.POINTER(ctypes.c_uint64)
i64p = ctypes.POINTER(ctypes.c_int64)


class ExitEvent(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_int32), ("exit_code", ctypes.c_int32), ("signal", ctypes.c_int32),
                ("core", ctypes.c_int32), ("ts_ns", ctypes.c_int64)]


# name -> (restype, argtypes)
SIGS = {
    "edl_sup_create": (vp, []),
    "edl_sup_spawn": (i32, [vp, cp, ctypes.POINTER(cp), ctypes.POINTER(cp), cp, cp, ctypes.POINTER(i32), i32, i32,
                            ctypes.POINTER(i32)]),
    "edl_sup_wait": (i32, [vp, i32, ctypes.POINTER(ExitEvent), i32]),
    "edl_sup_kill": (i32, [vp, i32, i32, i32]),
    "edl_sup_exiting": (i32, [vp, ctypes.POINTER(i32), i32]),
    "edl_sup_num_children": (i32, [vp]),
    "edl_sup_destroy": (None, [vp]),
    "edl_shm_open": (vp, [cp, u64, i32, i32]),
    "edl_shm_pin": (i32, [vp]),
    "edl_shm_data": (vp, [vp, i32]),
    "edl_shm_prefault": (i32, [vp, i32]),
    "edl_shm_slot_bytes": (u64, [vp]),
    "edl_shm_nslots": (i32, [vp]),
    "edl_shm_current": (i32, [vp]),
    "edl_shm_begin": (i32, [vp]),
    "edl_shm_commit": (i32, [vp, i32, i64, i64, u64, u64, cp]),
    "edl_shm_latest": (i32, [vp, i64p, i64p, u64p, u64p, cp, i32]),
    "edl_shm_slot_info": (i32, [vp, i32, i64p, i64p, u64p, u64p, cp, i32]),
    "edl_shm_close": (i32, [vp, i32]),
    "edl_shm_unlink": (i32, [cp]),
    "edl_shm_fd": (i32, [vp]),
    "edl_shm_reassign": (i32, [vp, cp]),
    "edl_shm_relink": (i32, [vp, cp]),
    "edl_ckpt_engine_create": (vp, [i32, u64, i32]),
    "edl_ckpt_snapshot": (i64, [vp, vp, i32, u64p, u64p, u64p, vp, i64, i64, i64, cp]),
    "edl_ckpt_fence": (i32, [vp, i64, vp]),
    "edl_ckpt_status": (i32, [vp, i64]),
    "edl_ckpt_wait": (i32, [vp, i64, i32]),
    "edl_ckpt_restore": (i32, [vp, i32, i32, u64p, u64p, u64p, vp]),
    "edl_ckpt_engine_destroy": (None, [vp]),
    "edl_ckpt_engine_staging": (i32, [vp, u64, i32, i32]),
    "edl_ckpt_engine_staged_stats": (None, [vp, ctypes.POINTER(ctypes.c_double)]),
    "edl_shm_pinned": (i32, [vp]),
    "edl_mark_open": (vp, [cp, i32, i32, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
    "edl_mark_close": (None, [vp, i32]),
    "edl_shm_populate_async": (i32, [vp, i32]),
    "edl_shm_populate_progress": (u64, [vp, u64p]),
    "edl_ckpt_restore_pipelined": (i32, [vp, i32, i32, u64p, u64p, u64p, vp, u64, i32]),
    "edl_ckpt_restore_pipelined2": (i32, [vp, i32, i32, u64p, u64p, u64p, vp, u64, i32, i32,
                                          ctypes.POINTER(ctypes.c_double)]),
    "edl_stream_create_cumask": (vp, [i32, ctypes.POINTER(ctypes.c_uint32), i32, i32]),
    "edl_stream_destroy": (i32, [vp]),
    "edl_stream_get_cumask": (i32, [vp, ctypes.POINTER(ctypes.c_uint32), i32]),
    "edl_roctx_available": (i32, []),
    "edl_roctx_push": (i32, [cp]),
    "edl_roctx_pop": (i32, []),
    "edl_roctx_mark": (None, [cp]),
    "edl_xgmi_ws_create": (i32, [i32, u64, ctypes.POINTER(vp)]),
    "edl_xgmi_ws_handles": (i32, [vp, ctypes.c_char_p]),
    "edl_xgmi_ws_open": (i32, [vp, i32, i32, ctypes.c_char_p]),
    "edl_xgmi_ws_ptrs": (i32, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
    "edl_xgmi_ws_bytes": (u64, [vp]),
    "edl_xgmi_ws_abort_dev": (vp, [vp]),
    "edl_xgmi_ws_status_dev": (vp, [vp]),
    "edl_xgmi_ws_set_abort": (None, [vp, i32]),
    "edl_xgmi_ws_status": (i32, [vp]),
    "edl_xgmi_ws_destroy": (i32, [vp]),
    "edl_xgmi_ws_status_detail": (i32, [vp, ctypes.POINTER(i32)]),
    "edl_xgmi_buf_handle": (i32, [vp, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "edl_xgmi_buf_open": (i32, [i32, ctypes.c_char_p, ctypes.POINTER(vp)]),
    "edl_xgmi_buf_close": (i32, [i32, vp]),
}
