// TEST STUB -- not GLFW.  Declarations of the GLFW 3.4 calls the reference's examples make (the
// viewer window), for tests/test_examples_compile.py; defined in tests/cpp/stubs/mujoco_stub.cpp.
#pragma once

typedef struct GLFWwindow GLFWwindow;
typedef struct GLFWmonitor GLFWmonitor;

#ifdef __cplusplus
extern "C" {
#endif
int glfwInit(void);
void glfwTerminate(void);
GLFWwindow* glfwCreateWindow(int width, int height, const char* title, GLFWmonitor* monitor,
                             GLFWwindow* share);
void glfwMakeContextCurrent(GLFWwindow* window);
void glfwSwapInterval(int interval);
void glfwGetFramebufferSize(GLFWwindow* window, int* width, int* height);
void glfwSwapBuffers(GLFWwindow* window);
void glfwPollEvents(void);
#ifdef __cplusplus
}
#endif
