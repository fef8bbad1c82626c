// TEST STUB -- not MuJoCo.  Declarations of the MuJoCo 3.2.7 C API subset that the reference's
// examples/standing.cc and examples/walter_sr_standing.cc call (simulation + mjv/mjr viewer), so
// that those files compile UNCHANGED against include/operational-space-control/ in an image
// without MuJoCo (tests/test_examples_compile.py).  Struct fields: only the ones those files
// read; signatures as MuJoCo's public headers declare them.  tests/cpp/stubs/mujoco_stub.cpp
// defines every function (each reports failure) so the examples also LINK.
#pragma once

typedef double mjtNum;

typedef struct mjModel_ {
  mjtNum* key_qpos;
  mjtNum* key_qvel;
  mjtNum* key_ctrl;
} mjModel;

typedef struct mjData_ {
  mjtNum time;
  mjtNum* qpos;
  mjtNum* qvel;
  mjtNum* ctrl;
  mjtNum* qfrc_actuator;
} mjData;

typedef struct mjVFS_ mjVFS;

typedef struct mjvCamera_ { int type; } mjvCamera;
typedef struct mjvPerturb_ { int select; } mjvPerturb;
typedef struct mjvOption_ { int label; } mjvOption;
typedef struct mjvScene_ { int maxgeom; } mjvScene;
typedef struct mjrContext_ { int fontScale; } mjrContext;
typedef struct mjrRect_ { int left, bottom, width, height; } mjrRect;

typedef enum mjtCatBit_ { mjCAT_STATIC = 1, mjCAT_DYNAMIC = 2, mjCAT_DECOR = 4, mjCAT_ALL = 7 } mjtCatBit;
typedef enum mjtFontScale_ { mjFONTSCALE_50 = 50, mjFONTSCALE_100 = 100, mjFONTSCALE_150 = 150,
                             mjFONTSCALE_200 = 200, mjFONTSCALE_250 = 250, mjFONTSCALE_300 = 300 } mjtFontScale;

#ifdef __cplusplus
extern "C" {
#endif
mjModel* mj_loadXML(const char* filename, const mjVFS* vfs, char* error, int error_sz);
mjData* mj_makeData(const mjModel* m);
void mj_forward(const mjModel* m, mjData* d);
void mj_step(const mjModel* m, mjData* d);
void mj_resetDataKeyframe(const mjModel* m, mjData* d, int key);
void mj_deleteData(mjData* d);
void mj_deleteModel(mjModel* m);
void mjv_defaultCamera(mjvCamera* cam);
void mjv_defaultPerturb(mjvPerturb* pert);
void mjv_defaultOption(mjvOption* opt);
void mjv_defaultScene(mjvScene* scn);
void mjv_makeScene(const mjModel* m, mjvScene* scn, int maxgeom);
void mjv_freeScene(mjvScene* scn);
void mjv_updateScene(const mjModel* m, mjData* d, const mjvOption* opt, const mjvPerturb* pert,
                     mjvCamera* cam, int catmask, mjvScene* scn);
void mjr_defaultContext(mjrContext* con);
void mjr_makeContext(const mjModel* m, mjrContext* con, int fontscale);
void mjr_freeContext(mjrContext* con);
void mjr_render(mjrRect viewport, mjvScene* scn, const mjrContext* con);
#ifdef __cplusplus
}
#endif
