/*
 * jni.h -- a minimal JNI interface for compiling and exercising the JNI shim
 * (src/native/srtp_mi355x/SrtpMi355x.c) without a JDK.  TEST INFRASTRUCTURE:
 * the image has no JDK, so tests/jni_stub/fakejvm.c implements these calls over
 * a toy object model (byte/int/object arrays and RawPacket objects) and the
 * tests drive the shim's exported JNI functions through it (tests/test_jni_shim.py).
 *
 * Written from the JNI specification's function names and signatures (the
 * subset the shim uses); the function table is not laid out like a real
 * JNINativeInterface, so a library built against it runs only under
 * fakejvm.c, never in a JVM.
 */
#ifndef SRTP_TEST_JNI_STUB_H
#define SRTP_TEST_JNI_STUB_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct fj_obj *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jobjectArray;
typedef struct fj_field *jfieldID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    jsize (*GetArrayLength)(JNIEnv *env, jarray a);
    void (*GetIntArrayRegion)(JNIEnv *env, jintArray a, jsize start, jsize len, jint *buf);
    void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray a, jsize start, jsize len, jbyte *buf);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray a, jsize start, jsize len, const jbyte *buf);
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jfieldID (*GetFieldID)(JNIEnv *env, jclass c, const char *name, const char *sig);
    jobject (*GetObjectField)(JNIEnv *env, jobject o, jfieldID f);
    jint (*GetIntField)(JNIEnv *env, jobject o, jfieldID f);
    void (*SetIntField)(JNIEnv *env, jobject o, jfieldID f, jint v);
    void (*SetObjectField)(JNIEnv *env, jobject o, jfieldID f, jobject v);
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray a, jsize i);
    void (*SetObjectArrayElement)(JNIEnv *env, jobjectArray a, jsize i, jobject v);
    jint (*PushLocalFrame)(JNIEnv *env, jint capacity);
    jobject (*PopLocalFrame)(JNIEnv *env, jobject result);
    jbyteArray (*NewByteArray)(JNIEnv *env, jsize len);
    jint *(*GetIntArrayElements)(JNIEnv *env, jintArray a, jboolean *is_copy);
    void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray a, jint *elems, jint mode);
    void (*SetIntArrayRegion)(JNIEnv *env, jintArray a, jsize start, jsize len, const jint *buf);
    void (*ExceptionClear)(JNIEnv *env);
};

#endif
