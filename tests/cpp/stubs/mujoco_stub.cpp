// TEST STUB -- definitions behind tests/cpp/stubs/{mujoco,GLFW,rules_cc} so the reference's
// examples LINK against libosc_controller unchanged.  Nothing here simulates: mj_loadXML fails
// (the example then prints the error and returns 1) and every other call does nothing.
#include <cstdio>

#include "GLFW/glfw3.h"
#include "mujoco/mujoco.h"
#include "rules_cc/cc/runfiles/runfiles.h"

extern "C" {
mjModel* mj_loadXML(const char* filename, const mjVFS*, char* error, int error_sz) {
  if (error && error_sz > 0) std::snprintf(error, error_sz, "stub: no MuJoCo to load %s", filename);
  return nullptr;
}
mjData* mj_makeData(const mjModel*) { return nullptr; }
void mj_forward(const mjModel*, mjData*) {}
void mj_step(const mjModel*, mjData*) {}
void mj_resetDataKeyframe(const mjModel*, mjData*, int) {}
void mj_deleteData(mjData*) {}
void mj_deleteModel(mjModel*) {}
void mjv_defaultCamera(mjvCamera*) {}
void mjv_defaultPerturb(mjvPerturb*) {}
void mjv_defaultOption(mjvOption*) {}
void mjv_defaultScene(mjvScene*) {}
void mjv_makeScene(const mjModel*, mjvScene*, int) {}
void mjv_freeScene(mjvScene*) {}
void mjv_updateScene(const mjModel*, mjData*, const mjvOption*, const mjvPerturb*, mjvCamera*, int,
                     mjvScene*) {}
void mjr_defaultContext(mjrContext*) {}
void mjr_makeContext(const mjModel*, mjrContext*, int) {}
void mjr_freeContext(mjrContext*) {}
void mjr_render(mjrRect, mjvScene*, const mjrContext*) {}
int glfwInit(void) { return 0; }
void glfwTerminate(void) {}
GLFWwindow* glfwCreateWindow(int, int, const char*, GLFWmonitor*, GLFWwindow*) { return nullptr; }
void glfwMakeContextCurrent(GLFWwindow*) {}
void glfwSwapInterval(int) {}
void glfwGetFramebufferSize(GLFWwindow*, int* w, int* h) { *w = *h = 0; }
void glfwSwapBuffers(GLFWwindow*) {}
void glfwPollEvents(void) {}
}

namespace rules_cc::cc::runfiles {
Runfiles* Runfiles::Create(const std::string&, const std::string&, std::string*) {
  return new Runfiles;
}
std::string Runfiles::Rlocation(const std::string& path) const { return path; }
}  // namespace rules_cc::cc::runfiles
